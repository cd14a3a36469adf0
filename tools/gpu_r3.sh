set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_blaslt_epilogue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_lt.log 2>&1
echo "lt exit=$?" >> gpurun_out/r3_lt.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_lt.log 2>&1 && \
DPA_LT_GELU=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_nolt.log 2>&1
echo "exit=$?"
