# r4ab: the bench's in-process reference schedule (after the fused run) with / without the side-stream nll.
set -o pipefail
mkdir -p gpurun_out/r4ab
for i in 1 2; do
  for v in 1 0; do
    DPA_NLL_SIDE=$v timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --json-out gpurun_out/r4ab/b_${v}_$i.json > gpurun_out/r4ab/b_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4ab/b_${v}_$i.json'));print('nll_side=$v fused', d['ms_per_step'], 'ref', d['reference_schedule']['ms_per_step'])" | tee -a gpurun_out/r4ab/summary.txt
  done
done
