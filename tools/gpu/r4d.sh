# r4d: DiffuSeq-XL HBM headroom; graphed reference schedule with the deferred wgrads on the
# backward stream at forward caps 0 / 192; then PMC passes on the L = 128 attention kernels.
set -o pipefail
bash tools/gpu/xl_mem.sh || exit $?
mkdir -p gpurun_out/gab5
run() {
  env $2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --ref-windows 2 $3 \
    --json-out gpurun_out/gab5/$1.json > gpurun_out/gab5/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['reference_schedule'];print(sys.argv[2], d['ms_per_step'], r['ms_per_step'], r.get('hip_graph'), r.get('windows_ms'), [w.get('host_ms_per_step') for w in r.get('windows_diag',[])])" gpurun_out/gab5/$1.json $1 | tee -a gpurun_out/gab5/summary.txt
}
run graph_noside_cap0 "DPA_WGRAD_SIDE_STREAM=0 DPA_OVERLAP_FWD_CAP=0" "--ref-graph 1" && \
run graph_noside_cap192 "DPA_WGRAD_SIDE_STREAM=0 DPA_OVERLAP_FWD_CAP=192" "--ref-graph 1" && \
run eager_noside "DPA_WGRAD_SIDE_STREAM=0" "--ref-graph 0" && \
bash tools/gpu/pmc_a128.sh
echo "exit=$?"
