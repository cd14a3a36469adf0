#!/bin/bash
# Round 2: headline bench + kernel-trace profile after the fused input/residual LN,
# then the GPT-2 and seq512 configs (fused schedule only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2e_bench.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r2e_prof -o run -- python bench.py --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/r2e_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python tools/prof_summary.py /tmp/r2e_prof 60 6 > gpurun_out/r2e_prof_summary.txt 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --ref-steps 0 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --json-out gpurun_out/r2e_gpt2.json > gpurun_out/r2e_gpt2.log 2>&1 || { echo "gpt2 failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --ref-steps 0 --seq-len 512 --batch-size 512 --microbatch 64 \
  --json-out gpurun_out/r2e_seq512.json > gpurun_out/r2e_seq512.log 2>&1 || { echo "seq512 failed"; exit 1; }
echo ok
