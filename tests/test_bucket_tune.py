"""Measured bucket sizes (DDPEngine(bucket_cap_mb=0), parallel/ddp.py tune_bucket_sizes):
every rank takes the same decision from MAX-reduced timings, the cap is one of the swept sizes
and leaves at least min_buckets buckets, and world 1 keeps the fixed defaults.  gloo, CPU."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port
from distributed_pipeline_amd.parallel.ddp import DDPEngine, tune_bucket_sizes


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap, first, table = tune_bucket_sizes(16 * (1 << 20), sizes_mb=(0.25, 0.5, 1, 2), iters=2)
        torch.manual_seed(rank)
        model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 256))
        eng = DDPEngine(model, bucket_cap_mb=0, first_bucket_mb=0)
        q.put((rank, cap, first, [r["mb"] for r in table], eng.bucket_cap_mb, eng.first_bucket_mb,
               len(eng.buckets), eng.bucket_tune is not None))
    finally:
        dist.destroy_process_group()


def test_tuned_bucket_sizes_agree_across_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, cap0, first0, sizes0, ecap0, efirst0, nb0, tuned0), (_, cap1, first1, sizes1, ecap1, efirst1, nb1, tuned1) = res
    assert (cap0, first0, sizes0) == (cap1, first1, sizes1)  # one decision for all ranks
    assert cap0 in sizes0 and first0 in sizes0 and first0 <= cap0
    assert (ecap0, efirst0, nb0) == (ecap1, efirst1, nb1) and tuned0 and tuned1
    # the 0.75 MiB model: the cap is limited to a quarter of the gradients (>= 4 buckets),
    # floored at the smallest swept size
    assert ecap0 <= max(2.0, 0.75 / 4) and efirst0 <= ecap0


def test_world_one_keeps_defaults():
    assert tune_bucket_sizes(1 << 20) == (32.0, 4.0, None)
    eng = DDPEngine(torch.nn.Linear(8, 8), bucket_cap_mb=0, first_bucket_mb=0)
    assert (eng.bucket_cap_mb, eng.first_bucket_mb, eng.bucket_tune) == (32.0, 4.0, None)
