# r4s: 128-wide weight gradients zero-padded onto the 256 x 256 split-K kernel: GEMM tests, headline A/B
# (DPA_WGRAD_PAD=1 vs 0, interleaved), kernel stats.
set -o pipefail
mkdir -p gpurun_out/r4s
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_kernels.py tests/test_model_gpu.py > gpurun_out/r4s/tests.log 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    DPA_WGRAD_PAD=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4s/bench_${v}_$i.json > gpurun_out/r4s/bench_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4s/bench_${v}_$i.json'));print('pad=$v', d['ms_per_step'])" | tee -a gpurun_out/r4s/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/r4s/prof.log 2>&1 || exit $?
