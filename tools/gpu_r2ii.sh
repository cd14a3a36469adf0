# GPT-2 kernel profile with the fused row CE (summary on the box).
set -o pipefail
mkdir -p gpurun_out/r2ii
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2ii -o run -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 --data-workers 0 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/r2ii/prof.log 2>&1 &&
python tools/prof_summary.py /tmp/r2ii/run_results.db 30 4 > gpurun_out/r2ii/gpt2.stats.txt
echo "exit=$?"
