#!/bin/bash
# Round-2 rocprofv3 evidence: trace (steady-state k_sweep summary) + FETCH/WRITE PMC per config
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
TAG=r02_c2_f32 CONFIG=c2 XS=f32 B=512 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02_c3_f32 CONFIG=c3 XS=f32 B=128 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02_c4_f32 CONFIG=c4 XS=f32 B=128 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02_c2_2bit CONFIG=c2 XS=2bit B=512 ALG=12508000000 bash scripts/gpu_profile.sh || exit 1
TAG=r02_c5rank_f32 CONFIG=c5 XS=f32 B=512 ALG=250000000000 BENCH_ARGS="--P 125000" bash scripts/gpu_profile.sh || exit 1
