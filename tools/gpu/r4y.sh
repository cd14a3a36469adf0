# r4y: fast tanh in the activation epilogues: act / GEMM / model tests, kernel stats (compare with bench_kernel_stats_r4d.txt).
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_norm_act_kernels.py tests/test_gemm_kernels.py tests/test_model_gpu.py > gpurun_out/r4y/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new; do
  if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4y/prof_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/r4y/prof_$v.log 2>&1 || exit $?
done
