# Round check of the working tree on one MI355X: GPU suite, smoke, headline bench, kernel stats.
set -o pipefail
mkdir -p gpurun_out/chk
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/chk/gputests.log 2>&1
st=$?
echo "tests exit=$st" >> gpurun_out/chk/gputests.log
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/chk/bench.json > gpurun_out/chk/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/chk/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/chk/prof.log 2>&1
echo "exit=$?"
[ "$DPA_CHK_REFPROF" = 1 ] && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/chk/rprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 --exec-microbatch 64 > gpurun_out/chk/rprof.log 2>&1
echo "exit=$?"
