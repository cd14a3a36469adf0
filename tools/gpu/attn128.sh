# head_dim 128 attention: kernel numerics, model tests, DiffuSeq-XL + headline bench
mkdir -p gpurun_out/a128
timeout -k 10 300 python -u -m pytest tests/test_attention_kernel.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/a128/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 512 > gpurun_out/a128/xl.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/a128/bench.log 2>&1
