# r4l: fused-CE one-hot scatter: xent + model GPU tests, headline A/B (scatter on/off, interleaved).
set -o pipefail
mkdir -p gpurun_out/r4l
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r4l/tests.log 2>&1 || exit $?
for i in 1 2; do
  for s in 1 0; do
    DPA_XENT_ONEHOT_SCATTER=$s timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/r4l/bench_${s}_$i.json > gpurun_out/r4l/bench_${s}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4l/bench_${s}_$i.json'));print('scatter=$s', d['ms_per_step'])" | tee -a gpurun_out/r4l/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && DPA_XENT_ONEHOT_SCATTER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4l/prof -o run -- python3 bench.py --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/r4l/prof.log 2>&1 || exit $?
