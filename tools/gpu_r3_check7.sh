# LN (wide-row backward) + attention (uniform causal mask, general-path bias column sums) tests, then configs
set -o pipefail
mkdir -p gpurun_out/r7
timeout -k 10 400 python -u -m pytest tests/test_norm_act_kernels.py tests/test_attention_kernel.py tests/test_model_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r7/tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/r7/xl.json > gpurun_out/r7/xl.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --json-out gpurun_out/r7/gpt2.json > gpurun_out/r7/gpt2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 \
  --ref-steps 4 --json-out gpurun_out/r7/seq512.json > gpurun_out/r7/seq512.log 2>&1
echo "exit=$?"
