# Same-box A/B of the 256-B-row LDS swizzle: CE kernels + headline step, new (_C) vs old (_C_swzold).
set -o pipefail
mkdir -p gpurun_out/r2cc
for e in _C _C_swzold _C _C_swzold; do
  DPA_EXT=$e timeout -k 10 120 python tools/xent_bench.py > gpurun_out/r2cc/xent_$e.tmp 2>&1 || exit 1
  echo "$e $(grep '^{' gpurun_out/r2cc/xent_$e.tmp)" >> gpurun_out/r2cc/ab.txt
done
for e in _C _C_swzold _C _C_swzold; do
  DPA_EXT=$e timeout -k 10 300 python bench.py --steps 6 --warmup 2 --ref-steps 0 --json-out gpurun_out/r2cc/b.json > gpurun_out/r2cc/b.log 2>&1 || exit 1
  echo "$e bench $(python -c "import json; print(json.load(open('gpurun_out/r2cc/b.json'))['ms_per_step'])")" >> gpurun_out/r2cc/ab.txt
done
echo "exit=$?"
