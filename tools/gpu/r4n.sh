# r4n: lxent_dw per-logit rework (g in the exponent, one-hot only where a target hits the wave):
# xent tests, xent_bench new vs old (DPA_EXT=_C_ab = previous xent.hip), headline new vs old.
set -o pipefail
mkdir -p gpurun_out/r4n
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r4n/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/xent_bench.py >> gpurun_out/r4n/xent_new.txt 2>&1 || exit $?
  DPA_EXT=_C_ab timeout -k 10 200 python3 tools/xent_bench.py >> gpurun_out/r4n/xent_old.txt 2>&1 || exit $?
done
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4n/bench_${v}_$i.json > gpurun_out/r4n/bench_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4n/bench_${v}_$i.json'));print('$v', d['ms_per_step'])" | tee -a gpurun_out/r4n/summary.txt
  done
done
