# r4v: decoder CE weight gradient on a side stream overlapping the transformer backward
# (DPA_XENT_DW_SIDE=1 vs 0): GPU tests with it on, headline A/B interleaved.
set -o pipefail
mkdir -p gpurun_out/r4v
DPA_XENT_DW_SIDE=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_overlap_gpu.py tests/test_graph_gpu.py tests/test_xent_kernel.py tests/test_convergence_gpu.py > gpurun_out/r4v/tests.log 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    DPA_XENT_DW_SIDE=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4v/bench_${v}_$i.json > gpurun_out/r4v/bench_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4v/bench_${v}_$i.json'));print('dw_side=$v', d['ms_per_step'])" | tee -a gpurun_out/r4v/summary.txt
  done
done
