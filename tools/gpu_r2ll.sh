# attn_item cleanup: attention numerics + causal microbench + GPT-2 step.
set -o pipefail
mkdir -p gpurun_out/r2ll
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_kernel.py tests/test_model_gpu.py > gpurun_out/r2ll/tests.log 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 > gpurun_out/r2ll/attn.jsonl 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2ll/gpt2.json > gpurun_out/r2ll/gpt2.log 2>&1
echo "exit=$?"
