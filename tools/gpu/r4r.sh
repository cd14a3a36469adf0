# r4r: wgrad split search up to 8 rounds (GPT-2 LM-head weight gradient: 2 -> 3 splits): GEMM tests,
# GPT-2 bench new vs old (DPA_EXT=_C_ab = previous gemm256.hip), interleaved.
set -o pipefail
mkdir -p gpurun_out/r4r
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_kernels.py tests/test_xent_kernel.py > gpurun_out/r4r/tests.log 2>&1 || exit $?
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
    timeout -k 10 240 python -u bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
      --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r4r/gpt2_${v}_$i.json > gpurun_out/r4r/gpt2_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4r/gpt2_${v}_$i.json'));print('gpt2 $v', d['ms_per_step'])" | tee -a gpurun_out/r4r/summary.txt
  done
done
