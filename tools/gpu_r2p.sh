# Clean kernel profiles: headline (fused schedule only), GPT-2 seq1024, DiffuSeq-XL.
set -o pipefail
mkdir -p gpurun_out/r2p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/base -o run -- python3 bench.py --steps 5 --warmup 1 --ref-steps 0 > gpurun_out/r2p/base.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/gpt2 -o run -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/r2p/gpt2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/xl -o run -- python3 bench.py --steps 2 --warmup 1 --ref-steps 0 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 > gpurun_out/r2p/xl.log 2>&1
rc=$?; echo "exit=$rc"
for c in base gpt2 xl; do python tools/prof_summary.py gpurun_out/r2p/$c/run_results.db 40 > gpurun_out/r2p/$c.stats.txt 2>&1; done
rm -rf gpurun_out/r2p/base gpurun_out/r2p/gpt2 gpurun_out/r2p/xl
