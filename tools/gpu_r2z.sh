# Same-box A/B of the tile-starved split-K path (DPA_GEMM_SPLITK) on the reference schedule.
set -o pipefail
mkdir -p gpurun_out/r2z
for v in 0 1 0 1; do
  DPA_GEMM_SPLITK=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 --json-out gpurun_out/r2z/ref_$v.json > gpurun_out/r2z/ref_$v.log 2>&1 || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r2z/ref_$v.json')); print('splitk=$v', d['ms_per_step'])" >> gpurun_out/r2z/ab.txt
done
echo "exit=$?"
