# r4z: executed micro-batch size on the headline (whole batch 2048 vs 2 x 1024), interleaved.
set -o pipefail
mkdir -p gpurun_out/r4z
for i in 1 2; do
  for e in 0 1024; do
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --ref-steps 0 --exec-microbatch $e --json-out gpurun_out/r4z/b_${e}_$i.json > gpurun_out/r4z/b_${e}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4z/b_${e}_$i.json'));print('exec=$e', d['ms_per_step'], d['config']['exec_microbatch'])" | tee -a gpurun_out/r4z/summary.txt
  done
done
