# r4w: second-box confirmation of the side-stream nll (DPA_NLL_SIDE 1 vs 0, interleaved x2).
set -o pipefail
mkdir -p gpurun_out/r4w
for i in 1 2; do
  for v in 1 0; do
    DPA_NLL_SIDE=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4w/bench_${v}_$i.json > gpurun_out/r4w/bench_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4w/bench_${v}_$i.json'));print('nll_side=$v', d['ms_per_step'])" | tee -a gpurun_out/r4w/summary.txt
  done
done
