#!/bin/bash
# Round 2: full GPU suite + full-size convergence (bf16 native vs fp32 reference, 200 steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2l_pytest_gpu.log 2>&1
echo "pytest gpu exit=$?"
export DPA_CONVERGENCE_LOG=gpurun_out/convergence_base_r2b.log
timeout -k 10 900 python -u -m pytest tests/test_convergence_base_gpu.py -x -v -s --timeout 800 --timeout-method thread > gpurun_out/r2l_conv.log 2>&1
echo "convergence exit=$?"
