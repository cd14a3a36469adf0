# DiffuSeq-XL HBM headroom: auto executed micro-batch without / with the 8 GB reserve, and a
# fixed 3-chunk (704-sample) executed micro-batch; allocator retries and headroom at peak.
set -o pipefail
mkdir -p gpurun_out/xlm
x() {  # name "ENV=V" "args"
  env $2 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
    --microbatch 64 --ref-steps 0 $3 --json-out gpurun_out/xlm/$1.json > gpurun_out/xlm/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['ms_per_step'], d['config']['exec_microbatch'], 'peak', d.get('peak_hbm_gb'), 'headroom', d.get('hbm_headroom_at_peak_gb'), 'retries', d.get('alloc_retries'))" gpurun_out/xlm/$1.json $1 | tee -a gpurun_out/xlm/summary.txt
}
x auto "DPA_X=0" "" && x exec704 "DPA_X=0" "--exec-microbatch 704" && x auto_reserve8 "DPA_HBM_RESERVE_GB=8" ""
echo "exit=$?"
