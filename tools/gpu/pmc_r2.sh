# PMC pass (own run, kernel-trace only): MFMA busy share and LDS bank conflicts per kernel,
# headline step and GPT-2 step (fused schedule only).  bench prints warmup progress on
# stderr into the log under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d /tmp/pmc -o run -- python3 bench.py --steps 1 --warmup 1 --ref-steps 0 --data-workers 0 > gpurun_out/pmc2/run.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmc 20 > gpurun_out/pmc2/summary_base.txt &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d /tmp/pmcg -o run -- python3 bench.py --steps 1 --warmup 1 --ref-steps 0 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 --data-workers 0 > gpurun_out/pmc2/run_gpt2.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmcg 20 > gpurun_out/pmc2/summary_gpt2.txt
echo "exit=$?"
