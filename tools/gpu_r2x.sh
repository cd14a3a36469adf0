# Reference-schedule kernel profile after the small-T fixes (summary written on the box).
set -o pipefail
mkdir -p gpurun_out/r2x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2x_ref -o run -- python3 bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 --data-workers 0 > gpurun_out/r2x/ref.log 2>&1
rc=$?
python tools/prof_summary.py /tmp/r2x_ref/run_results.db 40 4 > gpurun_out/r2x/ref.stats.txt 2>&1
echo "exit=$rc"
