# r4f: L = 128 attention backward rework + GPT-2 head rework: attention / xent GPU tests, the
# attention micro-bench, the headline bench, then the GPT-2 head A/B and profile (r4e.sh).
set -o pipefail
mkdir -p gpurun_out/r4f
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_kernel.py tests/test_model_gpu.py > gpurun_out/r4f/tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/r4f/attn128.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4f/bench.json > gpurun_out/r4f/bench.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r4f/bench.json'));print('headline', d['ms_per_step'])" | tee gpurun_out/r4f/summary.txt
bash tools/gpu/r4e.sh
