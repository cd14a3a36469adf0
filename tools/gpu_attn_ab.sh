# attention microbenchmark A/B: online single-pass (default) vs two-pass forward
mkdir -p gpurun_out/ab
for tp in 0 1; do
  DPA_ATTN_TWOPASS=$tp timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 >> gpurun_out/ab/attn.jsonl 2>&1 || exit 1
  DPA_ATTN_TWOPASS=$tp timeout -k 10 120 python tools/attn_bench.py --B 512 --H 16 --L 128 --D 128 --p 0.1 >> gpurun_out/ab/attn.jsonl 2>&1 || exit 1
  DPA_ATTN_TWOPASS=$tp timeout -k 10 120 python tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 >> gpurun_out/ab/attn.jsonl 2>&1 || exit 1
done
