#!/bin/bash
# Round 2: PMC counters of the GEMM lab kernels (wgrad TR/TR main loop vs row-form main loop)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd tools/gemm_lab
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d /tmp/pmc_lab -o run -- ./gemm_lab 1 > ../../gpurun_out/r2k_lab.log 2>&1 || { echo "pmc failed"; exit 1; }
cd ../..
python tools/pmc_summary.py /tmp/pmc_lab 12 > gpurun_out/r2k_pmc.txt 2>&1
echo ok
