# attention with register-prefetched tiles (fwd online + both bwd kernels): numerics, microbench, model benches
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests/test_attention_kernel.py tests/test_model_gpu.py tests/test_bert_golden.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pf/tests.log 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 128 --H 12 --L 1024 --causal --p 0.1 > gpurun_out/pf/attn.jsonl 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 512 --H 16 --L 128 --D 128 --p 0.1 >> gpurun_out/pf/attn.jsonl 2>&1 &&
timeout -k 10 120 python tools/attn_bench.py --B 512 --H 12 --L 512 --p 0.1 >> gpurun_out/pf/attn.jsonl 2>&1 &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/pf/gpt2.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 > gpurun_out/pf/seq512.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 512 > gpurun_out/pf/xl.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/pf/bench.log 2>&1
