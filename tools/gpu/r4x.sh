# r4x: reference 32 x 64 schedule with / without the side-stream nll (DPA_NLL_SIDE), interleaved.
set -o pipefail
mkdir -p gpurun_out/r4x
for i in 1 2; do
  for v in 1 0; do
    DPA_NLL_SIDE=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --ref-steps 0 --exec-microbatch 64 --json-out gpurun_out/r4x/ref_${v}_$i.json > gpurun_out/r4x/ref_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4x/ref_${v}_$i.json'));print('ref nll_side=$v', d['ms_per_step'])" | tee -a gpurun_out/r4x/summary.txt
  done
done
