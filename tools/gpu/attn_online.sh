# single-pass (online softmax) attention forward: numerics + A/B against the two-pass kernel
mkdir -p gpurun_out/ao
timeout -k 10 300 python -u -m pytest tests/test_attention_kernel.py tests/test_model_gpu.py tests/test_bert_golden.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ao/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/ao/gpt2_online.log 2>&1 &&
DPA_ATTN_TWOPASS=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/ao/gpt2_twopass.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --seq-len 512 --batch-size 512 --microbatch 64 > gpurun_out/ao/seq512_online.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 512 > gpurun_out/ao/xl_online.log 2>&1
