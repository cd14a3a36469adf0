# Causal bwd back to one instance; LN bwd spill-free at D = 2048: numerics, microbench, GPT-2 / XL steps.
set -o pipefail
mkdir -p gpurun_out/r2r
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_kernel.py tests/test_norm_act_kernels.py > gpurun_out/r2r/tests.log 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 >> gpurun_out/r2r/attn.jsonl 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 512 --H 16 --L 128 --D 128 --p 0.1 >> gpurun_out/r2r/attn.jsonl 2>&1 &&
DPA_ATTN_TWOPASS=1 timeout -k 10 120 python tools/attn_bench.py --B 512 --H 16 --L 128 --D 128 --p 0.1 >> gpurun_out/r2r/attn_twopass.jsonl 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2r/gpt2.json > gpurun_out/r2r/gpt2.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/r2r/xl.json > gpurun_out/r2r/xl.log 2>&1
echo "exit=$?"
