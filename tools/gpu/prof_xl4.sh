# rocprofv3 kernel stats of DiffuSeq-XL (BASELINE #5) with the auto executed micro-batch; summarised on the box.
set -o pipefail
mkdir -p gpurun_out/xl4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_xl4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
  --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --ref-steps 0 > gpurun_out/xl4/prof.log 2>&1 || exit $?
f=$(ls /tmp/prof_xl4/run_kernel_stats.csv /tmp/prof_xl4/*/*/run_kernel_stats.csv 2>/dev/null | head -1)
python tools/prof_summary.py "$f" 40 2 > gpurun_out/xl4/summary.txt 2>&1
echo "exit=$?"
