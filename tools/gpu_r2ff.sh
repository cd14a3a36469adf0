# Fused CE forward with half the targets ignored (sorted last) vs none.
set -o pipefail
mkdir -p gpurun_out/r2ff
timeout -k 10 120 python tools/xent_bench.py > gpurun_out/r2ff/xent.jsonl 2>&1 &&
timeout -k 10 120 python tools/xent_bench.py --ignore-frac 0.5 >> gpurun_out/r2ff/xent.jsonl 2>&1
echo "exit=$?"
