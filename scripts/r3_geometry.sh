#!/bin/bash
# round 3: streaming geometry knobs (row-range alignment, streaming workgroup cap) on the driver's window
LS_VARIANTS="${GEO_VARIANTS:-def:: al32::BRR_ROW_ALIGN=32 wg200::BRR_STREAM_WG=200 def2:: al32b::BRR_ROW_ALIGN=32 wg200b::BRR_STREAM_WG=200}" \
  bash "$(dirname "$0")/r3_lagswitch.sh"
