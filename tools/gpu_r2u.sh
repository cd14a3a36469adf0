# Split-K wgrad merge A/B: atomics only / workspace forced / cost model; then the gemm tests.
set -o pipefail
mkdir -p gpurun_out/r2u
DPA_WGRAD_WS=0 timeout -k 10 180 python tools/wgrad_bench.py >> gpurun_out/r2u/wgrad.jsonl 2>&1 &&
DPA_WGRAD_WS=1 timeout -k 10 180 python tools/wgrad_bench.py >> gpurun_out/r2u/wgrad.jsonl 2>&1 &&
timeout -k 10 180 python tools/wgrad_bench.py >> gpurun_out/r2u/wgrad.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_kernels.py > gpurun_out/r2u/tests.log 2>&1
echo "exit=$?"
