# Reference 32 x 64 schedule: eager vs HIP-graph replay (default runtime, and with the runtime's
# packet-capture replay off, DEBUG_CLR_GRAPH_PACKET_CAPTURE=0), 2 windows of 8 steps each; then
# DiffuSeq-XL (auto executed micro-batch) for the HBM headroom after settling.
set -o pipefail
mkdir -p gpurun_out/gab
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_overlap_multirank_gpu.py tests/test_graph_gpu.py > gpurun_out/gab/tests.log 2>&1 || exit $?
run() {  # name "ENV=V ..." "bench args"
  env $2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --ref-windows 2 $3 \
    --json-out gpurun_out/gab/$1.json > gpurun_out/gab/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['reference_schedule'];print(sys.argv[2], d['ms_per_step'], r['ms_per_step'], r.get('hip_graph'), r.get('windows_ms'), [{k:v for k,v in w.items() if k.startswith('host')} for w in r.get('windows_diag',[])])" gpurun_out/gab/$1.json $1 | tee -a gpurun_out/gab/summary.txt
}
run eager "DPA_X=0" "--ref-graph 0" && \
run graph "DPA_X=0" "--ref-graph 1" && \
run graph_nopc "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--ref-graph 1" && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/gab/xl.json > gpurun_out/gab/xl.log 2>&1
echo "exit=$?"
