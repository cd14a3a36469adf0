# r4e: GPT-2 LM-head changes (MALL-sized forward chunks, all-token dx GEMM): xent GPU tests, then
# GPT-2 small bench interleaved new / old (DPA_XENT_FWD_CHUNK_MB=2048 DPA_XENT_DX_ALL=0), then
# a GPT-2 kernel profile.
set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xent_kernel.py > gpurun_out/g2/tests.log 2>&1 || exit $?
g() {  # name "ENV=V ..."
  env $2 timeout -k 10 240 python -u bench.py --steps 4 --warmup 2 --model gpt2 --config-name gpt2 --seq-len 1024 \
    --batch-size 128 --microbatch 16 --ref-steps 0 --json-out gpurun_out/g2/$1.json > gpurun_out/g2/$1.log 2>&1 || return $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['ms_per_step'], d.get('peak_hbm_gb'))" gpurun_out/g2/$1.json $1 | tee -a gpurun_out/g2/summary.txt
}
g new1 "DPA_X=0" && g old1 "DPA_XENT_FWD_CHUNK_MB=2048 DPA_XENT_DX_ALL=0" && g new2 "DPA_X=0" && g old2 "DPA_XENT_FWD_CHUNK_MB=2048 DPA_XENT_DX_ALL=0" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g2/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --model gpt2 --config-name gpt2 --seq-len 1024 --batch-size 128 --microbatch 16 --ref-steps 0 > gpurun_out/g2/prof.log 2>&1
echo "exit=$?"
