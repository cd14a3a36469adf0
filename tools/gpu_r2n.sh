# RCCL at world 2 on one GPU (both ranks on cuda:0), then the bench's DDP path at N=2,
# then the reference 32x64 schedule alone under rocprof (kernel time vs wall).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 tools/probes/rccl_two_ranks.py > gpurun_out/rccl2.log 2>&1
echo "probe exit=$?" >> gpurun_out/rccl2.log
if grep -q "allreduce 3.0" gpurun_out/rccl2.log; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29532 bench.py --gpus 2 --steps 5 --warmup 2 --batch-size 512 --ref-steps 0 > gpurun_out/bench2.log 2>&1
  echo "bench2 exit=$?" >> gpurun_out/bench2.log
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profref -o run -- python3 bench.py --steps 3 --warmup 1 --exec-microbatch 64 --ref-steps 0 > gpurun_out/profref.log 2>&1
echo "profref exit=$?"
