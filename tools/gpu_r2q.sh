# Mask-free specialisation of full attention tiles: numerics + microbench, then the profiles.
set -o pipefail
mkdir -p gpurun_out/r2q
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_kernel.py > gpurun_out/r2q/tests.log 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 >> gpurun_out/r2q/attn.jsonl 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 >> gpurun_out/r2q/attn.jsonl 2>&1 &&
bash tools/gpu_r2p.sh
