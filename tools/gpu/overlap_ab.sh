# Reference-schedule A/B: weight-gradient side stream and forward-stream grid cap in the overlapped
# micro-batch schedule (plus the overlap/deferral GPU tests).
set -o pipefail
mkdir -p gpurun_out/ovl
timeout -k 10 300 python -u -m pytest tests/test_overlap_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ovl/tests.log 2>&1 || exit $?
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --ref-steps 8 --json-out gpurun_out/ovl/$tag.json > gpurun_out/ovl/$tag.log 2>&1 || return $?
  python -c "import json;d=json.load(open('gpurun_out/ovl/$tag.json'));print('$tag', d['reference_schedule']['ms_per_step'])"
}
for r in 1 2 3; do
  run base_r$r DPA_WGRAD_SIDE_STREAM=0 || exit $?
  run side_r$r DPA_WGRAD_SIDE_STREAM=1 || exit $?
  run side_cap160_r$r DPA_WGRAD_SIDE_STREAM=1 DPA_OVERLAP_FWD_CAP=160 || exit $?
  run side_cap192_r$r DPA_WGRAD_SIDE_STREAM=1 DPA_OVERLAP_FWD_CAP=192 || exit $?
done
