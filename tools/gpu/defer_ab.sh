# Reference-schedule A/B of the weight-gradient deferral depth (DPA_DEFER_WGRAD), plus the new GPU tests.
set -o pipefail
mkdir -p gpurun_out/defer
timeout -k 10 600 python -u -m pytest tests/test_gemm_kernels.py tests/test_overlap_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/defer/tests.log 2>&1 || exit $?
for r in 1 2; do
  for d in 0 2 4; do
    DPA_DEFER_WGRAD=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --ref-steps 4 --json-out gpurun_out/defer/b_d${d}_r${r}.json > gpurun_out/defer/b_d${d}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/defer/b_d${d}_r${r}.json'));print('depth $d', d['ms_per_step'], d['reference_schedule'])"
  done
done
