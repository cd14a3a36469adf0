set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_norm_act_kernels.py tests/test_overlap_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 \
  --microbatch 64 --ref-steps 0 --json-out gpurun_out/r5/xl.json > gpurun_out/r5/xl.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/s512ref -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --ref-steps 0 --seq-len 512 --batch-size 512 --microbatch 64 --exec-microbatch 64 > gpurun_out/r5/s512ref.log 2>&1
echo "exit=$?"
