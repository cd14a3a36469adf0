# PMC pass on the general attention kernels: causal L=1024 vs non-causal L=512 (instruction
# mix and waits per kernel).  Short program; hard time limit per pass.
set -o pipefail
mkdir -p gpurun_out/pmca
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  --kernel-trace --output-format csv -d /tmp/pmca -o run -- python3 tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 > gpurun_out/pmca/causal.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmca 8 > gpurun_out/pmca/causal_summary.txt 2>&1
[ $rc -eq 0 ] || { echo "exit=$rc"; exit $rc; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  --kernel-trace --output-format csv -d /tmp/pmcb -o run -- python3 tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 > gpurun_out/pmca/noncausal.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmcb 8 > gpurun_out/pmca/noncausal_summary.txt 2>&1
echo "exit=$rc"
