# PMC passes on the L = 128, D = 64 attention kernels of the headline (B = 2048, H = 12, p = 0.1):
# instruction mix / waits, then memory traffic.  Short program; hard time limit per pass.
set -o pipefail
mkdir -p gpurun_out/pmc128
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/pmc128/bench.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  --kernel-trace --output-format csv -d /tmp/pmc128a -o run -- python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/pmc128/a.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmc128a 8 > gpurun_out/pmc128/mix_summary.txt 2>&1
[ $rc -eq 0 ] || { echo "exit=$rc"; exit $rc; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY \
  --kernel-trace --output-format csv -d /tmp/pmc128b -o run -- python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/pmc128/b.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmc128b 8 > gpurun_out/pmc128/fetch_summary.txt 2>&1
[ $rc -eq 0 ] || { echo "exit=$rc"; exit $rc; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_WAVES \
  --kernel-trace --output-format csv -d /tmp/pmc128c -o run -- python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/pmc128/c.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmc128c 8 > gpurun_out/pmc128/write_summary.txt 2>&1
echo "exit=$rc"
