# Dynamic GEMM tile queue (DPA_GEMMP_DYNAMIC) on the overlapped reference schedules, interleaved same-box A/B.
set -o pipefail
mkdir -p gpurun_out/dyn
for r in 1 2; do
  for d in 0 1; do
    DPA_GEMMP_DYNAMIC=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --ref-steps 3 --ref-windows 2 --json-out gpurun_out/dyn/b_d${d}_r${r}.json > gpurun_out/dyn/b_d${d}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/dyn/b_d${d}_r${r}.json'));r=d['reference_schedule'];print('seq128 dyn $d', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
    DPA_GEMMP_DYNAMIC=$d timeout -k 10 300 python bench.py --steps 2 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 3 --ref-windows 2 --json-out gpurun_out/dyn/s_d${d}_r${r}.json > gpurun_out/dyn/s_d${d}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/dyn/s_d${d}_r${r}.json'));r=d['reference_schedule'];print('seq512 dyn $d', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
  done
done
