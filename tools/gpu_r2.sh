set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
echo "pytest exit=$?" >> gpurun_out/r2_pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 64 --microbatch 16 --exec-microbatch 16 --steps 5 --warmup 2 > gpurun_out/r2_bench_gpt2.log 2>&1
echo "exit=$?"
