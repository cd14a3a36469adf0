# Reference-schedule run-to-run spread: several processes, each timing several windows, for grid caps on
# the forward stream's persistent GEMMs (DPA_OVERLAP_FWD_CAP) x hardware queues per process, interleaved.
set -o pipefail
mkdir -p gpurun_out/refvar
for r in 1 2 3; do
  for q in 4 8; do
    for cap in 0 128; do
      GPU_MAX_HW_QUEUES=$q DPA_OVERLAP_FWD_CAP=$cap timeout -k 10 300 python bench.py --steps 1 --warmup 1 --ref-steps 3 --ref-windows 4 --json-out gpurun_out/refvar/q${q}c${cap}_r${r}.json > gpurun_out/refvar/q${q}c${cap}_r${r}.log 2>&1 || exit $?
      python -c "import json;d=json.load(open('gpurun_out/refvar/q${q}c${cap}_r${r}.json'));r=d['reference_schedule'];print('q $q cap $cap', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
    done
  done
done
