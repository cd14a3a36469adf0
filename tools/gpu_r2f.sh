#!/bin/bash
# Round 2: kernel profiles of the secondary configs (GPT-2 seq1024, DiffuSeq seq512, DiffuSeq-XL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2f_gpt2 -o run -- python bench.py --steps 2 --warmup 1 --ref-steps 0 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/r2f_gpt2.log 2>&1 || { echo "gpt2 failed"; exit 1; }
python tools/prof_summary.py /tmp/r2f_gpt2 40 3 > gpurun_out/r2f_gpt2_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2f_s512 -o run -- python bench.py --steps 2 --warmup 1 --ref-steps 0 --seq-len 512 --batch-size 512 --microbatch 64 > gpurun_out/r2f_s512.log 2>&1 || { echo "s512 failed"; exit 1; }
python tools/prof_summary.py /tmp/r2f_s512 40 3 > gpurun_out/r2f_s512_summary.txt 2>&1
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --ref-steps 0 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --json-out gpurun_out/r2f_xl.json > gpurun_out/r2f_xl.log 2>&1 || { echo "xl failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r2f_xlp -o run -- python bench.py --steps 1 --warmup 1 --ref-steps 0 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 > gpurun_out/r2f_xlp.log 2>&1 || { echo "xl prof failed"; exit 1; }
python tools/prof_summary.py /tmp/r2f_xlp 40 2 > gpurun_out/r2f_xl_summary.txt 2>&1
echo ok
