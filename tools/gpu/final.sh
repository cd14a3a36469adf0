# Round-end style check of HEAD: full GPU suite, smoke, headline bench (+ reference schedule).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/final/gputests.log 2>&1
echo "tests exit=$?" >> gpurun_out/final/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/final/bench.json > gpurun_out/final/bench.log 2>&1
echo "exit=$?"
