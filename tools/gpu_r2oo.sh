# Full-size GPT-2 small bf16-native vs fp32-torch loss curves, 200 steps (BASELINE config #4 numerics).
set -o pipefail
mkdir -p gpurun_out/r2oo
timeout -k 10 900 python tools/convergence_gpt2.py --steps 200 --out gpurun_out/r2oo/convergence_gpt2.log > gpurun_out/r2oo/run.log 2>&1
echo "exit=$?"
