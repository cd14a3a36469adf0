# Full-size DiffuSeq-base seq512 bf16-native vs fp32-torch loss curves, 200 steps (BASELINE config #3 numerics).
set -o pipefail
mkdir -p gpurun_out/r2pp
timeout -k 10 1000 python tools/convergence_diffuseq.py --seq-len 512 --batch 128 --steps 200 --seed 11 --out gpurun_out/r2pp/convergence_seq512_s11.log > gpurun_out/r2pp/run.log 2>&1
echo "exit=$?"
