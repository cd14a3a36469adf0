# New attention cases (XCD-interleaved order), headline bench, secondary configs.
set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_kernel.py > gpurun_out/r2s/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/r2s/base.json > gpurun_out/r2s/base.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 0 \
  --json-out gpurun_out/r2s/seq512.json > gpurun_out/r2s/seq512.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2s/gpt2.json > gpurun_out/r2s/gpt2.log 2>&1
echo "exit=$?"
