# attention A/B in one call: DPA_EXT=_C_ab (tools/ab_variant.py build of an older attention.hip) vs the
# current _C, interleaved, on the GPT-2 causal shape, XL's L=128 D=128 and seq512's L=512.
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for ext in _C_ab _C; do
    DPA_EXT=$ext timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 | sed "s/^/$ext r$r /" >> gpurun_out/ab/attn.jsonl || exit 1
    DPA_EXT=$ext timeout -k 10 120 python tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 | sed "s/^/$ext r$r /" >> gpurun_out/ab/attn.jsonl || exit 1
  done
done
grep -h fwd_TF gpurun_out/ab/attn.jsonl
