# New 256-B-row LDS swizzle: numerics (xent, gemm, attention), CE + D=128 attention microbench,
# PMC bank conflicts of the CE kernels.
set -o pipefail
mkdir -p gpurun_out/r2bb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xent_kernel.py tests/test_gemm_kernels.py tests/test_attention_kernel.py > gpurun_out/r2bb/tests.log 2>&1 &&
timeout -k 10 120 python tools/xent_bench.py >> gpurun_out/r2bb/xent.jsonl 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 512 --H 16 --L 128 --D 128 --p 0.1 >> gpurun_out/r2bb/attn.jsonl 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d /tmp/pmcx -o run -- python3 tools/xent_bench.py > gpurun_out/r2bb/pmc.log 2>&1 &&
python tools/pmc_summary.py /tmp/pmcx 8 > gpurun_out/r2bb/pmc_summary.txt
echo "exit=$?"
