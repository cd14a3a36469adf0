# Round check with the output-based LayerNorm backward: full GPU suite, smoke, interleaved
# A/B of DPA_LN_SAVE_OUT (0 = h copy, 1 = output-based), kernel stats of the headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lnc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/lnc/gputests.log 2>&1
st=$?
echo "tests exit=$st" >> gpurun_out/lnc/gputests.log
[ $st -eq 0 ] || exit $st
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/lnc/smoke.log 2>&1 || exit 3
for i in 0 1 2 3 4 5; do
  if [ $((i % 2)) -eq 0 ]; then V=0; else V=1; fi
  DPA_LN_SAVE_OUT=$V timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 --json-out gpurun_out/lnc/bench_$i.json > gpurun_out/lnc/ab_$i.log 2>&1 || exit 4
  echo "DPA_LN_SAVE_OUT=$V $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d.get("peak_hbm_gb"))' gpurun_out/lnc/bench_$i.json)" | tee -a gpurun_out/lnc/ab.txt
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/lnc/bench_full.json > gpurun_out/lnc/bench_full.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lnc/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/lnc/prof.log 2>&1
echo "prof exit=$?"
