# Column-sum deferral (ops/nn.py _WgradDeferral.ln_part / bias_part): interleaved same-box A/B of
# DPA_DEFER_COLSUM on the reference 32 x 64 schedule (forward-stream cap at its default).
set -o pipefail
mkdir -p gpurun_out/colsum
for r in 1 2 3; do
  for c in 0 1; do
    DPA_DEFER_COLSUM=$c timeout -k 10 300 python bench.py --steps 1 --warmup 1 --ref-steps 3 --ref-windows 3 --json-out gpurun_out/colsum/b_c${c}_r${r}.json > gpurun_out/colsum/b_c${c}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/colsum/b_c${c}_r${r}.json'));r=d['reference_schedule'];print('colsum $c', d['ms_per_step'], r['ms_per_step'], r['windows_ms'])"
  done
done
