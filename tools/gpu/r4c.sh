# r4c: reference-schedule variants (one-stream deferral, graph, contention knobs) + lab small-token study.
set -o pipefail
mkdir -p gpurun_out/gab3
bash tools/gpu/graph_ab4.sh || exit $?
run() {
  env $2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --ref-windows 2 $3 \
    --json-out gpurun_out/gab3/$1.json > gpurun_out/gab3/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['reference_schedule'];print(sys.argv[2], d['ms_per_step'], r['ms_per_step'], r.get('hip_graph'), r.get('windows_ms'), [w.get('host_ms_per_step') for w in r.get('windows_diag',[])])" gpurun_out/gab3/$1.json $1 | tee -a gpurun_out/gab3/summary.txt
}
run graph_cap64 "DPA_OVERLAP_FWD_CAP=64" "--ref-graph 1" && \
run graph_noside "DPA_WGRAD_SIDE_STREAM=0" "--ref-graph 1" && \
timeout -k 10 120 tools/gemm_lab/gemm_lab 5 small > gpurun_out/gab3/lab_small.txt 2>&1
echo "exit=$?"
