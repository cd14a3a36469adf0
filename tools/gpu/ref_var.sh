# Overlap/deferral GPU tests, then the reference-schedule run-to-run spread: processes x windows, with the
# host enqueue time per window (total, forwards, backwards).
set -o pipefail
mkdir -p gpurun_out/refvar
timeout -k 10 400 python -u -m pytest tests/test_overlap_gpu.py tests/test_model_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/refvar/tests.log 2>&1 || { tail -30 gpurun_out/refvar/tests.log; exit 1; }
tail -2 gpurun_out/refvar/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --ref-steps 3 --ref-windows 3 --json-out gpurun_out/refvar/h_r${r}.json > gpurun_out/refvar/h_r${r}.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/refvar/h_r${r}.json'));r=d['reference_schedule'];print(d['ms_per_step'], r['ms_per_step'], r['windows_ms'], [(w['host_ms_per_step'], w.get('host_fwd_ms_per_step'), w.get('host_bwd_ms_per_step')) for w in r['windows_diag']])"
done
cat /proc/loadavg
