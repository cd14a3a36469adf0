# r4g: general attention kernels (dropout template, store addressing): attention GPU tests, causal
# L = 1024 micro-bench, GPT-2 small bench x2, headline bench.
set -o pipefail
mkdir -p gpurun_out/r4g
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_kernel.py tests/test_model_gpu.py > gpurun_out/r4g/tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 > gpurun_out/r4g/attn_causal.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --B 2048 --H 12 --L 128 --p 0.1 > gpurun_out/r4g/attn128.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r4g/gpt2_$i.json > gpurun_out/r4g/gpt2_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4g/gpt2_$i.json'));print('gpt2', d['ms_per_step'])" | tee -a gpurun_out/r4g/summary.txt
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4g/bench.json > gpurun_out/r4g/bench.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r4g/bench.json'));print('headline', d['ms_per_step'])" | tee -a gpurun_out/r4g/summary.txt
