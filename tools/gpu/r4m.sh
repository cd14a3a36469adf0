# r4m: register-resident wide-vocabulary CE row kernel: xent tests, micro-bench A/B, GPT-2 bench A/B.
set -o pipefail
mkdir -p gpurun_out/r4m
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xent_kernel.py > gpurun_out/r4m/tests.log 2>&1 || exit $?
for r in 1 0 1 0; do
  DPA_XROWS_REG=$r timeout -k 10 120 python3 tools/xrows_bench.py >> gpurun_out/r4m/xrows.txt 2>&1 || exit $?
done
for i in 1 2; do
  for r in 1 0; do
    DPA_XROWS_REG=$r timeout -k 10 240 python -u bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
      --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r4m/gpt2_${r}_$i.json > gpurun_out/r4m/gpt2_${r}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4m/gpt2_${r}_$i.json'));print('gpt2 xrows_reg=$r', d['ms_per_step'])" | tee -a gpurun_out/r4m/summary.txt
  done
done
