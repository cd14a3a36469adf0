#!/bin/bash
# Round 2: GPT-2 seq1024 kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2g_gpt2 -o run -- python bench.py --steps 2 --warmup 1 --ref-steps 0 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/r2g_gpt2.log 2>&1 || { echo "gpt2 failed"; exit 1; }
python tools/prof_summary.py /tmp/r2g_gpt2 40 3 > gpurun_out/r2g_gpt2_summary.txt 2>&1
echo ok
