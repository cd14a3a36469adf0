# DiffuSeq-XL GEMM shapes (hipBLASLt vs native) and XL kernel profile after the D=128 attention
mkdir -p gpurun_out/xl
timeout -k 10 240 python tools/gemm_shapes_bench.py --tokens 65536 --hidden 2048 --native > gpurun_out/xl/gemm.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_xl -o run -- python3 bench.py --steps 1 --warmup 1 \
  --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 512 > gpurun_out/xl/prof.log 2>&1 &&
python tools/prof_summary.py /tmp/prof_xl/run_results.db 30 2 > gpurun_out/xl/prof_summary.txt &&
