# PMC passes (kernel trace only, one run per pass) on the forward / dgrad / weight-gradient GEMMs of one
# shape (tools/probes/gemm_pair.py): LDS instruction mix, bank conflicts, MFMA busy share.
set -o pipefail
mkdir -p gpurun_out/pmcwg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
  --kernel-trace --output-format csv -d /tmp/pmcwg_a -o run -- python3 tools/probes/gemm_pair.py > gpurun_out/pmcwg/a.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmcwg_a 6 > gpurun_out/pmcwg/a.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
  --kernel-trace --output-format csv -d /tmp/pmcwg_b -o run -- python3 tools/probes/gemm_pair.py > gpurun_out/pmcwg/b.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmcwg_b 6 > gpurun_out/pmcwg/b.txt 2>&1
echo "exit=$?"
