"""All-reduce bucket-size sweep: the data behind the DDP
engine's bucket sizes (4 MiB first bucket, then 32 MiB) on point-to-point xGMI.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29533 tools/bench_allreduce.py [--sizes-mb 1,4,16,32,64,128,256] [--dtype fp32]

One process per GPU over RCCL (torch backend "nccl"); ``--backend gloo`` runs the
same sweep on CPU ranks (plumbing check).  Prints one JSON line per size from
rank 0: time per all-reduce (max over ranks), algorithm bandwidth (bytes/time)
and bus bandwidth (algbw * 2(n-1)/n, the per-link load of a ring).
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None)
    a = ap.parse_args()
    backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        dist.init_process_group(backend, device_id=dev)
    else:
        dist.init_process_group(backend)
    dtype = torch.float32 if a.dtype == "fp32" else torch.bfloat16

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for mb in [float(s) for s in a.sizes_mb.split(",")]:
        n = max(1, int(mb * (1 << 20)) // torch.tensor([], dtype=dtype).element_size())
        x = torch.ones(n, dtype=dtype, device=dev)
        for _ in range(a.warmup):
            dist.all_reduce(x)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            dist.all_reduce(x)
        sync()
        dt = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64)
        dist.all_reduce(dt.to(dev) if backend == "nccl" else dt, op=dist.ReduceOp.MAX)
        sec = float(dt.item()) if backend != "nccl" else float(dt.to(dev).item())
        nbytes = n * x.element_size()
        algbw = nbytes / sec / 1e9
        if rank == 0:
            print(json.dumps({"backend": backend, "world": world, "dtype": a.dtype, "size_mb": mb,
                              "us": round(sec * 1e6, 1), "algbw_GBps": round(algbw, 2),
                              "busbw_GBps": round(algbw * 2 * (world - 1) / world, 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
