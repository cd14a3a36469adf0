# LN backward rows per block (A/B knob) on the reference 32 x 64 schedule.
set -o pipefail
mkdir -p gpurun_out/r2kk && rm -f gpurun_out/r2kk/ab.txt
for v in 4 32 4 32 16; do
  DPA_LN_BWD_MINROWS=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 --json-out gpurun_out/r2kk/r.json > gpurun_out/r2kk/r.log 2>&1 || exit 1
  echo "minrows=$v ref $(python -c "import json; print(json.load(open('gpurun_out/r2kk/r.json'))['ms_per_step'])")" >> gpurun_out/r2kk/ab.txt
done
echo "exit=0"
