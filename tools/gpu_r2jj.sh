# BASELINE config #3: DiffuSeq-base seq512 with the reference 8 x 64 no_sync schedule timed alongside the fused one.
set -o pipefail
mkdir -p gpurun_out/r2jj
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 3 \
  --json-out gpurun_out/r2jj/seq512.json > gpurun_out/r2jj/seq512.log 2>&1
echo "exit=$?"
