# r4k: L = 128 attention forward rework: attention + model GPU tests, micro-bench, headline x2.
set -o pipefail
mkdir -p gpurun_out/r4k
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_kernel.py tests/test_model_gpu.py > gpurun_out/r4k/tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/r4k/attn128.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4k/bench_$i.json > gpurun_out/r4k/bench_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4k/bench_$i.json'));print('headline', d['ms_per_step'])" | tee -a gpurun_out/r4k/summary.txt
done
