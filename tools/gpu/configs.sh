# Secondary BASELINE.json configs on one MI355X: seq512 (fused + its 8 x 64 reference schedule), GPT-2 small,
# DiffuSeq-XL (auto executed micro-batch).
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 \
  --ref-steps 4 --json-out gpurun_out/cfg/seq512.json > gpurun_out/cfg/seq512.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --json-out gpurun_out/cfg/gpt2.json > gpurun_out/cfg/gpt2.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/cfg/xl.json > gpurun_out/cfg/xl.log 2>&1
echo "exit=$?"
