#!/bin/bash
# Round-2 closing: C3/C4 rocprofv3 evidence, then the GPU suite, smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
EVIDENCE="c3_f32 c4_f32" bash scripts/gpu_evidence_r2d.sh || exit 1
bash scripts/gpu_final_r2.sh
