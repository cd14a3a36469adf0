# PMC passes on lxent_dw (new vs previous xent.hip via DPA_EXT=_C_ab): instruction mix, waits, LDS conflicts.
set -o pipefail
mkdir -p gpurun_out/pmcdw
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old; do
  if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU \
    --kernel-trace --output-format csv -d /tmp/pmcdw_a_$v -o run -- python3 tools/xent_bench.py > gpurun_out/pmcdw/a_$v.log 2>&1 || exit $?
  python tools/pmc_summary.py /tmp/pmcdw_a_$v 6 > gpurun_out/pmcdw/mix_$v.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-trace --output-format csv -d /tmp/pmcdw_b_$v -o run -- python3 tools/xent_bench.py > gpurun_out/pmcdw/b_$v.log 2>&1 || exit $?
  python tools/pmc_summary.py /tmp/pmcdw_b_$v 6 > gpurun_out/pmcdw/act_$v.txt 2>&1
done
echo done
