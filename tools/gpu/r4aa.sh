# r4aa: fused position / sequence sums of the input block's gradient: norm + model tests, kernel stats.
set -o pipefail
mkdir -p gpurun_out/r4aa
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_norm_act_kernels.py tests/test_model_gpu.py > gpurun_out/r4aa/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4aa/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/r4aa/prof.log 2>&1 || exit $?
