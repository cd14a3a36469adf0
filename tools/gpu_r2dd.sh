# Swizzle split (new XOR for W tiles / attention / gemm.hip TR, legacy for lxent_dw): numerics + CE bench + headline.
set -o pipefail
mkdir -p gpurun_out/r2dd
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xent_kernel.py tests/test_gemm_kernels.py tests/test_attention_kernel.py tests/test_model_gpu.py > gpurun_out/r2dd/tests.log 2>&1 &&
timeout -k 10 120 python tools/xent_bench.py > gpurun_out/r2dd/xent.jsonl 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/r2dd/base.json > gpurun_out/r2dd/base.log 2>&1
echo "exit=$?"
