#!/bin/bash
# A/B of an environment switch on the headline bench, interleaved on one box:
#   bash tools/gpu/ab.sh VAR VALUE_A VALUE_B [tests...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; shift 3
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread "$@" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; exit 1; }
fi
for i in 0 1 2 3; do
  if [ $((i % 2)) -eq 0 ]; then V=$A; else V=$B; fi
  env "$VAR=$V" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/ab_$i.log 2>&1 || { echo "bench $i failed"; exit 1; }
  echo "$VAR=$V $(tail -1 gpurun_out/ab_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
