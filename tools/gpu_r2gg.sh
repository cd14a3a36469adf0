# Config refresh with HEAD: headline kernel profile (summary on the box), seq512, GPT-2, XL.
set -o pipefail
mkdir -p gpurun_out/r2gg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2gg_base -o run -- python3 bench.py --steps 5 --warmup 1 --ref-steps 0 --data-workers 0 > gpurun_out/r2gg/base_prof.log 2>&1 &&
python tools/prof_summary.py /tmp/r2gg_base/run_results.db 40 6 > gpurun_out/r2gg/base.stats.txt &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 0 \
  --json-out gpurun_out/r2gg/seq512.json > gpurun_out/r2gg/seq512.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 \
  --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r2gg/gpt2.json > gpurun_out/r2gg/gpt2.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/r2gg/xl.json > gpurun_out/r2gg/xl.log 2>&1
echo "exit=$?"
