set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1_pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r1_bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r1_prof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/r1_prof.log 2>&1
echo "exit=$?"
