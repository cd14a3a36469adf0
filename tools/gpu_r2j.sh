#!/bin/bash
# Round 2: clean DiffuSeq-XL profile (exec micro-batch 1024 given explicitly: no OOM retry in the trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r2j_xl -o run -- python bench.py --steps 1 --warmup 1 --ref-steps 0 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 1024 > gpurun_out/r2j_xl.log 2>&1 || { echo "xl prof failed"; exit 1; }
python tools/prof_summary.py /tmp/r2j_xl 40 2 > gpurun_out/r2j_xl_summary.txt 2>&1
python tools/prof_summary.py /tmp/r2j_xl 60 2 --by-grid > gpurun_out/r2j_xl_by_grid.txt 2>&1
echo ok
