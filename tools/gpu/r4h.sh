# r4h: early aux prefetch of the DACT / residual dgrad epilogues: GEMM GPU tests, lab A/B
# (EARLY_AUX 0 / 1 builds interleaved), headline bench.
set -o pipefail
mkdir -p gpurun_out/r4h
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_kernels.py > gpurun_out/r4h/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 tools/gemm_lab/gemm_lab_m0 5 aux >> gpurun_out/r4h/lab_aux.txt 2>&1 || exit $?
  timeout -k 10 120 tools/gemm_lab/gemm_lab 5 aux >> gpurun_out/r4h/lab_aux.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4h/bench.json > gpurun_out/r4h/bench.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r4h/bench.json'));print('headline', d['ms_per_step'])" | tee gpurun_out/r4h/summary.txt
