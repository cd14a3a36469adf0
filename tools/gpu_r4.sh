set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_norm_act_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/r4_prof.log 2>&1
echo "exit=$?"
