# final4: round-end style check of HEAD (GPU suite, smoke, headline bench incl. reference schedule), then the
# side-stream nll A/B with the high-priority pool stream (in-process reference schedule).
set -o pipefail
mkdir -p gpurun_out/final4
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/final4/gputests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final4/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/final4/bench.json > gpurun_out/final4/bench.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/final4/bench.json'));print('default fused', d['ms_per_step'], 'ref', d['reference_schedule']['ms_per_step'])" | tee -a gpurun_out/final4/summary.txt
for v in 1 0; do
  DPA_NLL_SIDE=$v timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --json-out gpurun_out/final4/b_$v.json > gpurun_out/final4/b_$v.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/final4/b_$v.json'));print('nll_side=$v fused', d['ms_per_step'], 'ref', d['reference_schedule']['ms_per_step'])" | tee -a gpurun_out/final4/summary.txt
done
