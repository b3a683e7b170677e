#!/bin/bash
# Round-2 closing rocprofv3 evidence on the final kernels (profiles/r02c_*)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${EVIDENCE:-c2_f32 c2_2bit}; do
  case $c in
    c2_f32) TAG=r02c_c2_f32 CONFIG=c2 XS=f32 B=512 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1 ;;
    c2_2bit) TAG=r02c_c2_2bit CONFIG=c2 XS=2bit B=512 ALG=12508000000 bash scripts/gpu_profile.sh || exit 1 ;;
    c3_f32) TAG=r02c_c3_f32 CONFIG=c3 XS=f32 B=128 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1 ;;
    c4_f32) TAG=r02c_c4_f32 CONFIG=c4 XS=f32 B=128 ALG=200000000000 bash scripts/gpu_profile.sh || exit 1 ;;
  esac
done
