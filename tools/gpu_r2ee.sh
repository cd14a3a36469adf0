# 128-B-row LDS swizzle: numerics (new), then same-box A/B new (_C) vs old (_C_swzold) on the
# general attention kernels and the GPT-2 step.
set -o pipefail
mkdir -p gpurun_out/r2ee
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_kernel.py tests/test_gemm_kernels.py tests/test_model_gpu.py > gpurun_out/r2ee/tests.log 2>&1 || exit 1
for e in _C _C_swzold _C _C_swzold; do
  DPA_EXT=$e timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 > gpurun_out/r2ee/a.tmp 2>&1 || exit 1
  echo "$e causal $(grep '"causal"' gpurun_out/r2ee/a.tmp | tail -1)" >> gpurun_out/r2ee/ab.txt
  DPA_EXT=$e timeout -k 10 120 python tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 > gpurun_out/r2ee/a.tmp 2>&1 || exit 1
  echo "$e noncausal $(grep '"causal"' gpurun_out/r2ee/a.tmp | tail -1)" >> gpurun_out/r2ee/ab.txt
done
for e in _C _C_swzold; do
  DPA_EXT=$e timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2ee/g.json > gpurun_out/r2ee/g.log 2>&1 || exit 1
  echo "$e gpt2 $(python -c "import json; print(json.load(open('gpurun_out/r2ee/g.json'))['ms_per_step'])")" >> gpurun_out/r2ee/ab.txt
done
echo "exit=0"
