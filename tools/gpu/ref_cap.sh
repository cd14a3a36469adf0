# Forward-stream grid cap (DPA_OVERLAP_FWD_CAP) on the other overlapped reference schedules: seq512 8 x 64 and
# GPT-2 8 x 16, interleaved 0 vs 128.
set -o pipefail
mkdir -p gpurun_out/refcap
for r in 1 2; do
  for cap in 0 128; do
    DPA_OVERLAP_FWD_CAP=$cap timeout -k 10 300 python bench.py --steps 1 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 3 --ref-windows 2 --json-out gpurun_out/refcap/s_c${cap}_r${r}.json > gpurun_out/refcap/s_c${cap}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/refcap/s_c${cap}_r${r}.json'));r=d['reference_schedule'];print('seq512 cap $cap', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
    DPA_OVERLAP_FWD_CAP=$cap timeout -k 10 300 python bench.py --steps 1 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 --ref-steps 3 --ref-windows 2 --json-out gpurun_out/refcap/g_c${cap}_r${r}.json > gpurun_out/refcap/g_c${cap}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/refcap/g_c${cap}_r${r}.json'));r=d['reference_schedule'];print('gpt2 cap $cap', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
  done
done
