"""Time the fused linear-cross-entropy kernels at the DiffuSeq-base training shape.

    python tools/xent_bench.py [--N 262144] [--V 30522] [--E 128]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=262144)
    ap.add_argument("--V", type=int, default=30522)
    ap.add_argument("--E", type=int, default=128)
    ap.add_argument("--ignore-frac", type=float, default=0.0,
                    help="fraction of targets set to -100, sorted last (the logged masked nll)")
    a = ap.parse_args()
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    N, V, E = a.N, a.V, a.E
    x = torch.randn(N, E, device="cuda").bfloat16()
    W = (torch.randn(V, E, device="cuda") * 0.5).bfloat16()
    b = (torch.randn(V, device="cuda") * 0.1).bfloat16()
    tgt = torch.randint(0, V, (N,), device="cuda")
    if a.ignore_frac > 0:
        tgt[int(N * (1 - a.ignore_frac)):] = -100
    loss, lse = ext.lxent_fwd(x, W, b, tgt)
    dl = torch.rand(N, device="cuda")
    f = bench(lambda: ext.lxent_fwd(x, W, b, tgt))
    bw = bench(lambda: ext.lxent_bwd(dl, x, W, b, tgt, lse, True, True, True))
    dxo = bench(lambda: ext.lxent_bwd(dl, x, W, b, tgt, lse, True, False, False))
    dwo = bench(lambda: ext.lxent_bwd(dl, x, W, b, tgt, lse, False, True, True))
    fdx = bench(lambda: ext.lxent_fwd_dx(x, W, b, tgt)) if hasattr(ext, "lxent_fwd_dx") else None
    fl = 2.0 * N * V * E
    print(json.dumps({"N": N, "V": V, "E": E, "ignore_frac": a.ignore_frac, "fwd_ms": round(f, 3), "fwd_logit_TF": round(fl / f / 1e9, 1),
                      "bwd_ms": round(bw, 3), "dx_ms": round(dxo, 3), "dw_ms": round(dwo, 3),
                      "fused_fwd_dx_ms": round(fdx, 3) if fdx else None}))


if __name__ == "__main__":
    main()
