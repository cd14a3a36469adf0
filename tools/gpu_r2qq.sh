# DiffuSeq-XL kernel profile with HEAD (summary written on the box).
set -o pipefail
mkdir -p gpurun_out/r2qq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r2qq -o run -- python3 bench.py --steps 2 --warmup 1 --ref-steps 0 --data-workers 0 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 > gpurun_out/r2qq/xl.log 2>&1 &&
python tools/prof_summary.py /tmp/r2qq/run_results.db 30 > gpurun_out/r2qq/xl.stats.txt
echo "exit=$?"
