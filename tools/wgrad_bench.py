"""Split-K weight-gradient microbenchmark: dW[N][K] += dy[T][N]^T x[T][K] through
ext.gemm_wgrad for the DiffuSeq-base encoder shapes at the fused (T = 262144) and the
reference micro-batch (T = 8192) token counts.  Merge mode / split count come from
DPA_WGRAD_WS / DPA_WGRAD_SPLITS (read once per process).  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_pipeline_amd.ops._ext import get_ext  # noqa: E402

ext = get_ext(required=True)
SHAPES = [("qkv", 2304, 768), ("attn_out", 768, 768), ("ffn_in", 3072, 768), ("ffn_out", 768, 3072)]
for T in (8192, 262144):
    for name, N, K in SHAPES:
        dy = torch.randn(T, N, device="cuda").bfloat16()
        x = torch.randn(T, K, device="cuda").bfloat16()
        dW = torch.zeros(N, K, device="cuda")
        ext.gemm_wgrad(dy, x, dW, None)
        torch.cuda.synchronize()
        ref = dy[:4096].float().t() @ x[:4096].float() if T == 8192 else None
        reps = 50 if T == 8192 else 10
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ext.gemm_wgrad(dy, x, dW, None)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        err = None
        if T == 8192:  # numerics of one call on a half-length slice vs fp32
            d2 = torch.zeros(N, K, device="cuda")
            ext.gemm_wgrad(dy[:4096].contiguous(), x[:4096].contiguous(), d2, None)
            err = float((d2 - ref).abs().max() / ref.abs().max())
        # hipBLASLt yardstick: the same product, bf16 out (no fp32 accumulation into a gradient)
        dyt = dy.t()
        s.record()
        for _ in range(reps):
            torch.mm(dyt, x)
        e.record()
        torch.cuda.synchronize()
        us_bl = s.elapsed_time(e) / reps * 1e3
        print(json.dumps({"T": T, "shape": name, "N": N, "K": K, "us": round(us, 2),
                          "TF": round(2 * T * N * K / us / 1e6, 1), "blaslt_us": round(us_bl, 2),
                          "blaslt_TF": round(2 * T * N * K / us_bl / 1e6, 1), "relerr": err,
                          "ws": os.environ.get("DPA_WGRAD_WS", "model")}), flush=True)
        del dy, x, dW
