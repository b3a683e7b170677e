#!/bin/bash
# Round-2 rocprofv3 evidence after the f64 value tables, the Horseshoe chain call and the static ring
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
TAG=r02b_c2_2bit CONFIG=c2 XS=2bit B=512 ALG=12508000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02b_c4_f32 CONFIG=c4 XS=f32 B=128 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02b_c2_f32 CONFIG=c2 XS=f32 B=512 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
