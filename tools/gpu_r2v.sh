# wgrad workspace merge on by default: GEMM/model/trainer GPU tests, headline + reference schedule.
set -o pipefail
mkdir -p gpurun_out/r2v
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_kernels.py tests/test_model_gpu.py tests/test_bert_golden.py tests/test_ddp_engine.py tests/test_multirank_gpu.py > gpurun_out/r2v/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/r2v/base.json > gpurun_out/r2v/base.log 2>&1
echo "exit=$?"
