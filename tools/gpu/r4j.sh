# r4j: deferral depth 8 (multi-segment wgrad up to 8 segments): GEMM + overlap GPU tests, then the
# 32 x 64 reference schedule and seq512 8 x 64 at depth 4 vs 8 (interleaved), then the host profile.
set -o pipefail
mkdir -p gpurun_out/r4j
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_kernels.py tests/test_overlap_gpu.py > gpurun_out/r4j/tests.log 2>&1 || exit $?
for d in 4 8 4 8; do
  DPA_DEFER_WGRAD=$d timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --ref-steps 8 --json-out gpurun_out/r4j/ref_d$d.json > gpurun_out/r4j/ref_d$d.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4j/ref_d$d.json'));print('depth $d ref32x64', d['reference_schedule']['ms_per_step'])" | tee -a gpurun_out/r4j/summary.txt
done
for d in 4 8; do
  DPA_DEFER_WGRAD=$d timeout -k 10 300 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 \
    --ref-steps 4 --json-out gpurun_out/r4j/s512_d$d.json > gpurun_out/r4j/s512_d$d.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4j/s512_d$d.json'));print('depth $d seq512 fused', d['ms_per_step'], '8x64', d['reference_schedule']['ms_per_step'])" | tee -a gpurun_out/r4j/summary.txt
done
bash tools/gpu/host_prof.sh
