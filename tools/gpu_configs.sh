# Secondary BASELINE.json configs on one MI355X (3 timed steps each).
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 \
  --json-out gpurun_out/cfg/seq512.json > gpurun_out/cfg/seq512.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --json-out gpurun_out/cfg/gpt2.json > gpurun_out/cfg/gpt2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --exec-microbatch 512 --json-out gpurun_out/cfg/xl.json > gpurun_out/cfg/xl.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --reference-equivalent --seq-len 512 --batch-size 512 \
  --microbatch 64 --json-out gpurun_out/cfg/seq512_ref.json > gpurun_out/cfg/seq512_ref.log 2>&1
