"""GEMM efficiency at the reference schedule's micro-batch size (8192 tokens): the persistent
256 x 256 kernel, the 128 x 128 kernel (gemm.hip) and hipBLASLt, ms per call and TFLOP/s.

    python tools/probes/small_gemm.py [T]
"""
import json
import sys

import torch

from distributed_pipeline_amd.ops._ext import get_ext


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    ext = get_ext(required=True)
    torch.manual_seed(0)
    out = {}
    for N, K in ((768, 768), (768, 3072), (3072, 768), (2304, 768)):
        x = torch.randn(T, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        dy = torch.randn(T, N, device="cuda").bfloat16()
        fl = 2.0 * T * N * K
        r = {}
        for name, on, half in (("p256", True, 0), ("p128x256", True, 2), ("k128", False, 0)):
            ext.set_gemm256(on)
            ext.set_gemmp_half(half)
            r[f"fwd_{name}"] = timeit(lambda: ext.gemm_nt(x, W, b, 0))
            r[f"dgrad_{name}"] = timeit(lambda: ext.gemm_nn(dy, W))
            if on and N == 768:
                r[f"fwd_resdrop_{name}"] = timeit(lambda: ext.gemm_nt_res(x, W, b, dy, 0.1, 1, 2))
            if on and N >= 2304:
                r[f"fwd_gelu_q8_{name}"] = timeit(lambda: ext.gemm_nt(x, W, b, 1, 2))
        ext.set_gemm256(True)
        ext.set_gemmp_half(-1)
        r["fwd_blaslt"] = timeit(lambda: torch.addmm(b, x, W.t()))
        r["dgrad_blaslt"] = timeit(lambda: dy @ W)
        out[f"{T}x{N}x{K}"] = {k: (round(v * 1e3, 1), round(fl / v / 1e9, 0)) for k, v in r.items()}
        print(f"{T}x{N}x{K}", json.dumps(out[f"{T}x{N}x{K}"]), flush=True)
    print("us/call, TFLOP/s")


if __name__ == "__main__":
    main()
