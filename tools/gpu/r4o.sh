# r4o: CE row kernels write loss / lse slices in place (no per-chunk copies): xent tests, GPT-2 bench x2, profile.
set -o pipefail
mkdir -p gpurun_out/r4o
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xent_kernel.py tests/test_model_gpu.py > gpurun_out/r4o/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/r4o/gpt2_$i.json > gpurun_out/r4o/gpt2_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4o/gpt2_$i.json'));print('gpt2', d['ms_per_step'])" | tee -a gpurun_out/r4o/summary.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4o/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 --ref-steps 0 > gpurun_out/r4o/prof.log 2>&1 || exit $?
