# HIP-graph replay of the 32 x 64 reference schedule: is the captured multi-stream step
# executed with its streams concurrent?  Runtime knobs (DEBUG_HIP_FORCE_GRAPH_QUEUES with and
# without packet capture) + a short kernel trace of the graphed schedule for offline overlap
# analysis; then DiffuSeq-XL with the 8 GB HBM reserve the multi-GPU default applies.
set -o pipefail
mkdir -p gpurun_out/gab2
run() {  # name "ENV=V ..." "bench args"
  env $2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --ref-windows 2 $3 \
    --json-out gpurun_out/gab2/$1.json > gpurun_out/gab2/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['reference_schedule'];print(sys.argv[2], d['ms_per_step'], r['ms_per_step'], r.get('hip_graph'), r.get('windows_ms'), [w.get('host_ms_per_step') for w in r.get('windows_diag',[])])" gpurun_out/gab2/$1.json $1 | tee -a gpurun_out/gab2/summary.txt
}
run graph_q4 "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "--ref-graph 1" && \
run graph_q4_nopc "DEBUG_HIP_FORCE_GRAPH_QUEUES=4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--ref-graph 1" && \
run eager "DPA_X=0" "--ref-graph 0" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gab2/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --ref-steps 2 --ref-graph 1 > gpurun_out/gab2/trace.log 2>&1 && \
DPA_HBM_RESERVE_GB=8 timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/gab2/xl_reserve8.json > gpurun_out/gab2/xl_reserve8.log 2>&1
echo "exit=$?"
