# Fused wide-E row CE (forward leaves softmax - onehot in the kept logits): numerics, GPT-2 A/B.
set -o pipefail
mkdir -p gpurun_out/r2hh && rm -f gpurun_out/r2hh/ab.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r2hh/tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  DPA_XENT_ROWS_FUSED=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2hh/g.json > gpurun_out/r2hh/g.log 2>&1 || exit 1
  echo "fused=$v gpt2 $(python -c "import json; print(json.load(open('gpurun_out/r2hh/g.json'))['ms_per_step'])")" >> gpurun_out/r2hh/ab.txt
done
echo "exit=0"
