#!/bin/bash
# round 3: the adaptive pipeline lag's switch threshold (BRR_LAG_SWITCH, changed markers per block
# per 100,000 rows) on the driver's window, same box
VARIANTS="${LS_VARIANTS:-def:: ls12::BRR_LAG_SWITCH=12 ls15::BRR_LAG_SWITCH=15 def2:: ls12b::BRR_LAG_SWITCH=12 ls15b::BRR_LAG_SWITCH=15}" \
  bash "$(dirname "$0")/r3_variants.sh"
