# One-stream reference schedule with weight-gradient deferral (DPA_OVERLAP_MB=0), eager and as a
# replayed HIP graph, vs the overlapped eager default; the deferral GPU tests first.
set -o pipefail
mkdir -p gpurun_out/gab4
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_overlap_gpu.py > gpurun_out/gab4/tests.log 2>&1 || exit $?
run() {  # name "ENV=V ..." "bench args"
  env $2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --ref-windows 2 $3 \
    --json-out gpurun_out/gab4/$1.json > gpurun_out/gab4/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['reference_schedule'];print(sys.argv[2], d['ms_per_step'], r['ms_per_step'], r.get('hip_graph'), r.get('windows_ms'), [w.get('host_ms_per_step') for w in r.get('windows_diag',[])])" gpurun_out/gab4/$1.json $1 | tee -a gpurun_out/gab4/summary.txt
}
run eager_ovl "DPA_X=0" "--ref-graph 0" && \
run eager_seq "DPA_OVERLAP_MB=0" "--ref-graph 0" && \
run graph_seq "DPA_OVERLAP_MB=0" "--ref-graph 1" && \
run graph_ovl "DPA_X=0" "--ref-graph 1"
echo "exit=$?"
