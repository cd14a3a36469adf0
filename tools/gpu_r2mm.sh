# LM head: one wgrad GEMM over all kept chunks. Numerics + GPT-2 A/B vs the previous commit's behaviour
# is not switchable, so: tests, then GPT-2 twice.
set -o pipefail
mkdir -p gpurun_out/r2mm && rm -f gpurun_out/r2mm/ab.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r2mm/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2mm/g.json > gpurun_out/r2mm/g.log 2>&1 || exit 1
  echo "single-chunk gpt2 $(python -c "import json; print(json.load(open('gpurun_out/r2mm/g.json'))['ms_per_step'])")" >> gpurun_out/r2mm/ab.txt
done
echo "exit=0"
