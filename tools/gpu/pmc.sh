# PMC counters for the headline step (own run, kernel-trace only): MFMA busy share and LDS conflicts
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d /tmp/pmc -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmc/run.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmc 16 > gpurun_out/pmc/summary.txt
