# Same-box A/B: kept LM-head logits in one chunk vs 2 GiB chunks (GPT-2 step).
set -o pipefail
mkdir -p gpurun_out/r2nn && rm -f gpurun_out/r2nn/ab.txt
for v in 1 0 1 0; do
  DPA_XENT_SINGLE_CHUNK=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2nn/g.json > gpurun_out/r2nn/g.log 2>&1 || exit 1
  echo "single=$v gpt2 $(python -c "import json; print(json.load(open('gpurun_out/r2nn/g.json'))['ms_per_step'])")" >> gpurun_out/r2nn/ab.txt
done
echo "exit=0"
