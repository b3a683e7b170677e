#!/bin/bash
# which library variant crashes at process exit under rocprofv3 (small problem)
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in plain default; do
  if [ $v = plain ]; then export BRR_LIB=variants/libbrr_plain.so; else unset BRR_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/exit_$v -o run --output-format csv -- python3 bench.py --N 8192 --P 20000 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/exit_$v.log 2>&1
  echo "$v rc=$?"
done
timeout -k 10 120 python3 bench.py --N 8192 --P 20000 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/exit_noprof.log 2>&1; echo "noprof rc=$?"
exit 0
