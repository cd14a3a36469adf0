"""Debug: 2 ranks on one GPU (gloo), report which buckets disagree after finalize."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from basic_utils.dist_util import find_free_port  # noqa: E402

CFG = dict(model="diffuseq", config_name="tiny", hidden_size=256, num_layers=2, num_heads=4,
           intermediate_size=1024, vocab_size=3000, seq_len=128, hidden_dim=128, hidden_t_dim=128,
           dropout=0.0, precision=os.environ.get("PREC", "bf16"))


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
    from distributed_pipeline_amd.parallel.ddp import DDPEngine
    torch.manual_seed(1234 + rank)
    model = build_model(**CFG).cuda()
    eng = DDPEngine(model, shadow_dtype=torch.bfloat16 if CFG["precision"] == "bf16" else None,
                    bucket_cap_mb=1.0, first_bucket_mb=0.25)
    names = {id(p): n for n, p in model.named_parameters()}
    log = []
    orig = eng._launch

    def launch(b):
        log.append(("launch", b.index, [names[id(p)] for p in b.params if p.grad is None]))
        return orig(b)
    eng._launch = launch
    diff = create_gaussian_diffusion(steps=100)
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(1000, 3000, (world, 2, 4, 128), generator=g).cuda()
    mask = torch.ones_like(ids)
    mask[..., :32] = 0
    t = torch.randint(0, 100, (world, 2, 4), generator=g).cuda()
    eng.zero_grad()
    local = None
    for mb in range(2):
        ctx = eng.no_sync() if mb == 0 else torch.enable_grad()
        torch.manual_seed(99 + mb * 10 + rank)
        with ctx:
            terms = diff.training_losses(eng, None, t[rank, mb], dict(input_ids=ids[rank, mb], input_mask=mask[rank, mb]))
        terms["loss"].mean().backward()
    eng.finalize()
    torch.cuda.synchronize()
    ranges = [(b.index, b.start, b.end, [names[id(p)] for p in b.params]) for b in eng.buckets]
    q.put((rank, eng.space.grad_flat.cpu().numpy(), ranges, [x[:2] for x in log]))
    dist.destroy_process_group()


if __name__ == "__main__":
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda x: x[0])
    [p.join() for p in ps]
    g0, g1 = res[0][1], res[1][1]
    print("launch order r0:", res[0][3])
    print("launch order r1:", res[1][3])
    for idx, s, e, names in res[0][2]:
        d = np.abs(g0[s:e] - g1[s:e]).max()
        print(idx, s, e, f"maxdiff={d:.3e}", names[:6])
