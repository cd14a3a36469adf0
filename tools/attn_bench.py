"""Time the attention kernels at the DiffuSeq-base training shape (per layer call).

    python tools/attn_bench.py [--B 2048] [--H 12] [--L 128] [--p 0.1]
Set DPA_ATTN128=0 to time the generic (non-persistent) kernels instead.
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
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--D", type=int, default=64, help="head dim (64, or 128 for DiffuSeq-XL)")
    ap.add_argument("--causal", action="store_true", help="GPT-2 masking")
    a = ap.parse_args()
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    B, H, L, D, c = a.B, a.H, a.L, a.D, a.causal
    qkv = (torch.randn(B, L, 3 * H * D, device="cuda") * 0.5).bfloat16()
    # memory-pattern probes: contiguous copy vs per-head 128-B-segment gather
    gb = qkv.numel() * 2 * 2 / 1e9
    t_c = bench(lambda: qkv.clone())
    t_p = bench(lambda: qkv.view(B, L, 3, H, D).permute(0, 2, 3, 1, 4).contiguous())
    print(json.dumps({"copy_contig_GBps": round(gb / t_c * 1e3, 1),
                      "copy_head_gather_GBps": round(gb / t_p * 1e3, 1)}), flush=True)
    for p in sorted({0.0, a.p}):
        out, lse = ext.attn_fwd(qkv, H, p, c, 1, 0)
        dout = torch.randn_like(out)
        f = bench(lambda: ext.attn_fwd(qkv, H, p, c, 1, 0))
        b = bench(lambda: ext.attn_bwd(dout, qkv, out, lse, H, p, c, 1, 0))
        bdb = bench(lambda: ext.attn_bwd(dout, qkv, out, lse, H, p, c, 1, 0, True))
        gb_f = (qkv.numel() + out.numel()) * 2 / 1e9
        gb_b = (qkv.numel() * 2 + out.numel() * 2) * 2 / 1e9
        fl = 4.0 * B * H * L * L * D * (0.5 if c else 1.0)   # QK^T + PV
        print(json.dumps({"B": B, "H": H, "L": L, "D": D, "causal": c, "p": p,
                          "fwd_TF": round(fl / f / 1e9, 1), "bwd_TF": round(2.5 * fl / b / 1e9, 1),
                          "fwd_ms": round(f, 3), "fwd_GBps": round(gb_f / f * 1e3, 1),
                          "bwd_ms": round(b, 3), "bwd_GBps": round(gb_b / b * 1e3, 1),
                          "bwd_with_bias_colsum_ms": round(bdb, 3),
                          "fwd_us_per_item_per_cu": round(f * 1e3 / (B * H / 256), 2),
                          "bwd_us_per_item_per_cu": round(b * 1e3 / (B * H / 256), 2)}), flush=True)


if __name__ == "__main__":
    main()
