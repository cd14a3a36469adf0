# Vocabulary-split fused CE forward for small token counts: numerics, then the reference schedule.
set -o pipefail
mkdir -p gpurun_out/r2t
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r2t/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 --json-out gpurun_out/r2t/ref.json > gpurun_out/r2t/ref.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --ref-steps 0 --json-out gpurun_out/r2t/base.json > gpurun_out/r2t/base.log 2>&1
echo "exit=$?"
