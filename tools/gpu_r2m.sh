#!/bin/bash
# Round 2: GEMM first-iteration drain change - tests, then old/new lab binaries interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_kernels.py tests/test_model_gpu.py > gpurun_out/r2m_tests.log 2>&1 || { echo "tests failed"; exit 1; }
cd tools/gemm_lab
timeout -k 10 200 ./gemm_lab_old 3 > ../../gpurun_out/r2m_old1.txt 2>&1 || { echo "old lab failed"; exit 1; }
timeout -k 10 200 ./gemm_lab 3 > ../../gpurun_out/r2m_new1.txt 2>&1 || { echo "new lab failed"; exit 1; }
timeout -k 10 200 ./gemm_lab_old 3 > ../../gpurun_out/r2m_old2.txt 2>&1 || { echo "old lab failed"; exit 1; }
timeout -k 10 200 ./gemm_lab 3 > ../../gpurun_out/r2m_new2.txt 2>&1 || { echo "new lab failed"; exit 1; }
echo ok
