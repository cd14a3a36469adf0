"""Data-gradient GEMM dx = dy W through the transposed-B kernel (gemm_nn: W [N][K] read with
ds_read_b64_tr_b16) against the same product through the row-form forward kernel with a
transposed weight copy (gemm_nt(dy, W^T)): is a W^T shadow worth keeping?  T = 262144 tokens,
the DiffuSeq-base dgrad shapes; ms per call from HIP events, interleaved."""
import json

import torch

from distributed_pipeline_amd.ops._ext import get_ext


def timeit(fn, iters=10):
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
    ext = get_ext(required=True)
    torch.manual_seed(0)
    T = 262144
    out = {}
    for name, N, K in (("qkv", 2304, 768), ("attn_out", 768, 768), ("ffn_in", 3072, 768), ("ffn_out", 768, 3072)):
        dy = torch.randn(T, N, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
        WT = W.t().contiguous()
        a = ext.gemm_nn(dy, W)
        b = ext.gemm_nt(dy, WT, None, 0)[0]
        assert torch.equal(a, b) or (a.float() - b.float()).abs().max().item() < 1e-2
        r = {"nn_tr": [], "nt_rowform": []}
        for _ in range(3):
            r["nn_tr"].append(round(timeit(lambda: ext.gemm_nn(dy, W)), 4))
            r["nt_rowform"].append(round(timeit(lambda: ext.gemm_nt(dy, WT, None, 0)), 4))
        r["transpose_copy_ms"] = round(timeit(lambda: WT.copy_(W.t())), 4)
        out[name] = r
        print(name, json.dumps(r), flush=True)
        del dy, W, WT


if __name__ == "__main__":
    main()
