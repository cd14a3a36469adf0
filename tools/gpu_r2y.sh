# Split-K for tile-starved fwd/dgrad GEMMs: GEMM/model tests, reference schedule, headline.
set -o pipefail
mkdir -p gpurun_out/r2y
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_kernels.py tests/test_model_gpu.py tests/test_bert_golden.py tests/test_trainer.py > gpurun_out/r2y/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/r2y/base.json > gpurun_out/r2y/base.log 2>&1
echo "exit=$?"
