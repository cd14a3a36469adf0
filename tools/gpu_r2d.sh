#!/bin/bash
# Round 2: full-size numerics (DiffuSeq-base bf16 native vs fp32 reference, 200 steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export DPA_CONVERGENCE_LOG=gpurun_out/convergence_base_r2.log
timeout -k 10 900 python -u -m pytest tests/test_convergence_base_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r2d_conv.log 2>&1
echo "exit=$?"
