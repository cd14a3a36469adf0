# 128-tile wgrad split cap: GEMM tests, reference schedule.
set -o pipefail
mkdir -p gpurun_out/r2w
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_kernels.py tests/test_model_gpu.py > gpurun_out/r2w/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 --json-out gpurun_out/r2w/ref.json > gpurun_out/r2w/ref.log 2>&1
echo "exit=$?"
