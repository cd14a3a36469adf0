"""Probe: can two RCCL ranks share one HIP device on this pool?  Run under
torchrun --nproc-per-node 2; every rank binds cuda:0 (dist_util.dev() wraps
LOCAL_RANK around the visible devices).  Prints the all-reduce result."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from basic_utils import dist_util  # noqa: E402

dist_util.setup_dist()
r, w = dist.get_rank(), dist.get_world_size()
t = torch.full((1 << 20,), float(r + 1), device=dist_util.dev())
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {r}/{w} dev {dist_util.dev()} allreduce {t[0].item()} (expect {w * (w + 1) / 2})", flush=True)
dist_util.barrier()
dist.destroy_process_group()
