#!/bin/bash
# Round 2: persistent GEMM integration check - GEMM kernel tests, the full GPU suite,
# the headline bench and a kernel-trace profile of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_gemm_tests.log 2>&1 || { echo "gemm tests failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2a_bench.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a_prof -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/r2a_prof.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2a_pytest_gpu.log 2>&1
echo "pytest gpu exit=$?"
