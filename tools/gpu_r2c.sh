#!/bin/bash
# Round 2: direct-RCCL reducer + ZeRO reduce-scatter tests, bench with the reference schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 amd-smi topology --json > gpurun_out/r2c_topology.json 2>&1
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_gemm_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2c_bench.log 2>&1 || { echo "bench failed"; exit 1; }
echo ok
