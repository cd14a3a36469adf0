"""Time the exact GEMM calls the Linear op issues for DiffuSeq-base at a given token count:
fwd (addmm / mm), dgrad (dz @ W), wgrad (mm(dz^T, x, out_dtype=fp32)), per layer shape.
Optionally also the native MFMA GEMM kernels (--native)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20, warmup=5):
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
    ap.add_argument("--tokens", type=int, default=262144)
    ap.add_argument("--native", action="store_true")
    ap.add_argument("--hidden", type=int, default=768, help="2048 for DiffuSeq-XL")
    ap.add_argument("--ffn", type=int, default=0, help="default 4 x hidden")
    a = ap.parse_args()
    Hd = a.hidden
    F = a.ffn or 4 * Hd
    T = a.tokens
    dev = "cuda"
    shapes = [("qkv", Hd, 3 * Hd), ("attn_out", Hd, Hd), ("ffn_in", Hd, F), ("ffn_out", F, Hd)]
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    ext = None
    if a.native:
        from distributed_pipeline_amd.ops._ext import get_ext
        ext = get_ext(required=True)
    for name, K, N in shapes:
        x = torch.randn(T, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        dz = torch.randn(T, N, device=dev).bfloat16()
        gacc = torch.zeros(N, K, device=dev)
        f = bench(lambda: torch.addmm(b, x, w.t()))
        d = bench(lambda: dz @ w)
        g = bench(lambda: torch.mm(dz.t(), x, out_dtype=torch.float32))
        fl = 2.0 * T * K * N
        rec = {"name": name, "T": T, "K": K, "N": N,
               "fwd_ms": round(f, 3), "fwd_TF": round(fl / f / 1e9, 1),
               "dgrad_ms": round(d, 3), "dgrad_TF": round(fl / d / 1e9, 1),
               "wgrad_ms": round(g, 3), "wgrad_TF": round(fl / g / 1e9, 1)}
        if ext is not None and hasattr(ext, "gemm_wgrad"):
            def nat():
                ext.gemm_wgrad(dz, x, gacc, None)
            nw = bench(nat)
            ref = torch.mm(dz.t(), x, out_dtype=torch.float32)
            gacc.zero_()
            ext.gemm_wgrad(dz, x, gacc, None)
            err = (gacc - ref).abs().max().item() / ref.abs().max().item()
            gb = torch.zeros(N, device=dev)
            nwb = bench(lambda: ext.gemm_wgrad(dz, x, gacc, gb))
            rec.update(native_wgrad_ms=round(nw, 3), native_wgrad_TF=round(fl / nw / 1e9, 1),
                       native_wgrad_relerr=err, native_wgrad_with_db_ms=round(nwb, 3))
        if ext is not None and hasattr(ext, "gemm_nt"):
            nf = bench(lambda: ext.gemm_nt(x, w, b, 0))
            y = ext.gemm_nt(x, w, b, 0)[0]
            ref = torch.addmm(b, x, w.t()).float()
            rec.update(native_fwd_ms=round(nf, 3), native_fwd_TF=round(fl / nf / 1e9, 1),
                       native_fwd_relerr=((y.float() - ref).abs().max() / ref.abs().max()).item())
        if ext is not None and hasattr(ext, "gemm_nn"):
            nd = bench(lambda: ext.gemm_nn(dz, w))
            dxn = ext.gemm_nn(dz, w)
            ref = (dz @ w).float()
            rec.update(native_dgrad_ms=round(nd, 3), native_dgrad_TF=round(fl / nd / 1e9, 1),
                       native_dgrad_relerr=((dxn.float() - ref).abs().max() / ref.abs().max()).item())
        if ext is not None and name == "ffn_in":
            # fused-epilogue variants vs hipBLASLt + separate elementwise pass
            z = torch.randn(T, N, device=dev).bfloat16()
            dh = torch.randn(T, K, device=dev).bfloat16()   # grad arriving from ffn_out (width K)
            w2 = (torch.randn(K, N, device=dev) * 0.02).bfloat16()  # ffn_out weight [hidden, ffn]
            rec["gelu_fwd_native_ms"] = round(bench(lambda: ext.gemm_nt(x, w, b, 1)), 3)
            rec["gelu_fwd_blas_plus_eltwise_ms"] = round(bench(
                lambda: ext.bias_act_fwd(torch.mm(x, w.t()), b, 1)), 3)
            rec["dgelu_dgrad_native_ms"] = round(bench(lambda: ext.gemm_nn_dact(dh, w2, z, 1)), 3)
            rec["dgelu_dgrad_blas_plus_eltwise_ms"] = round(bench(
                lambda: ext.bias_act_bwd(dh @ w2, z, 1, False)), 3)
        for k in tot:
            tot[k] += rec[f"{k}_ms"]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"per_layer_ms": {k: round(v, 3) for k, v in tot.items()},
                      "x12_layers_ms": round(12 * sum(tot.values()), 2)}))


if __name__ == "__main__":
    main()
