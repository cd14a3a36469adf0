# r4q: LayerNorm dropout bits from a pair hash instead of Philox: norm / dropout / model / trainer GPU tests,
# kernel stats new vs old (DPA_EXT=_C_ab = previous norm.hip), headline bench new vs old.
set -o pipefail
mkdir -p gpurun_out/r4q
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dropout_hash.py tests/test_norm_act_kernels.py tests/test_model_gpu.py tests/test_attention_kernel.py > gpurun_out/r4q/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old; do
  if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4q/prof_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/r4q/prof_$v.log 2>&1 || exit $?
done
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DPA_EXT=_C_ab; else unset DPA_EXT; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4q/bench_${v}_$i.json > gpurun_out/r4q/bench_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4q/bench_${v}_$i.json'));print('$v', d['ms_per_step'])" | tee -a gpurun_out/r4q/summary.txt
  done
done
