# attention A/B + XL diagnosis (auto vs explicit executed micro-batch, kernel profile)
set -o pipefail
mkdir -p gpurun_out/r6
bash tools/gpu_attn_ab.sh > gpurun_out/r6/attn_ab.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --exec-microbatch 1024 --ref-steps 0 --json-out gpurun_out/r6/xl1024.json > gpurun_out/r6/xl1024.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/xlprof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --ref-steps 0 > gpurun_out/r6/xlprof.log 2>&1
echo "exit=$?"
