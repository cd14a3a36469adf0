# rocprofv3 kernel stats of the secondary configs (DiffuSeq-XL, GPT-2 small);
# summarised on the box (the rocpd databases are too large to copy back).
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_xl -o run -- python3 bench.py --steps 1 --warmup 1 \
  --config-name diffuseq-xl --batch-size 2048 --microbatch 64 --exec-microbatch 512 > gpurun_out/prof_xl.log 2>&1 &&
python tools/prof_summary.py /tmp/prof_xl/run_results.db 40 2 > gpurun_out/prof_xl_summary.txt &&
python tools/prof_summary.py /tmp/prof_xl/run_results.db 60 2 --by-grid > gpurun_out/prof_xl_grid.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_gpt2 -o run -- python3 bench.py --steps 2 --warmup 1 \
  --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 > gpurun_out/prof_gpt2.log 2>&1 &&
python tools/prof_summary.py /tmp/prof_gpt2/run_results.db 40 3 > gpurun_out/prof_gpt2_summary.txt
