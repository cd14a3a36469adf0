# Column-sum deferral (ops/nn.py _WgradDeferral.ln_part / bias_part): new GPU tests, then an
# interleaved same-box A/B of DPA_DEFER_COLSUM on the reference schedule (headline config and
# seq512's 8 x 64).
set -o pipefail
mkdir -p gpurun_out/colsum
timeout -k 10 600 python -u -m pytest tests/test_norm_act_kernels.py tests/test_overlap_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/colsum/tests.log 2>&1 || exit $?
tail -3 gpurun_out/colsum/tests.log
for r in 1 2; do
  for c in 0 1; do
    DPA_DEFER_COLSUM=$c timeout -k 10 300 python bench.py --steps 2 --warmup 1 --ref-steps 4 --json-out gpurun_out/colsum/b_c${c}_r${r}.json > gpurun_out/colsum/b_c${c}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/colsum/b_c${c}_r${r}.json'));print('colsum $c', d['ms_per_step'], d['reference_schedule'])"
  done
done
for r in 1 2; do
  for c in 0 1; do
    DPA_DEFER_COLSUM=$c timeout -k 10 300 python bench.py --steps 1 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 --ref-steps 3 --json-out gpurun_out/colsum/s_c${c}_r${r}.json > gpurun_out/colsum/s_c${c}_r${r}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/colsum/s_c${c}_r${r}.json'));print('seq512 colsum $c', d['ms_per_step'], d['reference_schedule'])"
  done
done
