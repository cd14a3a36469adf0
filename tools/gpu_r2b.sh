#!/bin/bash
# Round 2: headline step under different executed micro-batch sizes (reference schedule = 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for emb in 64 256 1024 2048; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --exec-microbatch $emb > gpurun_out/r2b_bench_emb$emb.log 2>&1 || { echo "bench $emb failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b_prof64 -o run -- python bench.py --steps 2 --warmup 1 --exec-microbatch 64 > gpurun_out/r2b_prof64.log 2>&1
echo done
