"""Micro-benchmark of the epilogue variants at the headline shapes (T = 262144 tokens, BERT-base
widths): ms per call from HIP events, interleaved A/B pairs on identical inputs.

    python tools/probes/epi_bench.py [T]
"""
import json
import sys

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
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    ext = get_ext(required=True)
    torch.manual_seed(0)
    H, F = 768, 3072
    dev = "cuda"
    x = torch.randn(T, H, device=dev).bfloat16()
    W1 = (torch.randn(F, H, device=dev) * 0.03).bfloat16()
    b1 = torch.randn(F, device=dev).bfloat16() * 0.1
    W2 = (torch.randn(H, F, device=dev) * 0.03).bfloat16()
    b2 = torch.randn(H, device=dev).bfloat16() * 0.1
    Wo = (torch.randn(H, H, device=dev) * 0.03).bfloat16()
    g = torch.ones(H, device=dev).bfloat16()
    be = torch.zeros(H, device=dev).bfloat16()
    res = {}
    _, z16, _ = ext.gemm_nt(x, W1, b1, 1, 1)
    _, z8, _ = ext.gemm_nt(x, W1, b1, 1, 2)
    dy = torch.randn(T, H, device=dev).bfloat16()
    for rep in range(2):
        res.setdefault("ffn_in_fwd_bf16_act", []).append(timeit(lambda: ext.gemm_nt(x, W1, b1, 1, 1)))
        res.setdefault("ffn_in_fwd_u8_act", []).append(timeit(lambda: ext.gemm_nt(x, W1, b1, 1, 2)))
        res.setdefault("ffn_out_dgrad_dact_bf16", []).append(timeit(lambda: ext.gemm_nn_dact(dy, W2, z16, 4, True)))
        res.setdefault("ffn_out_dgrad_dact_u8", []).append(timeit(lambda: ext.gemm_nn_dact(dy, W2, z8, 5, True)))
        res.setdefault("attn_out_fwd_plain", []).append(timeit(lambda: ext.gemm_nt(x, Wo, b2, 0)))
        res.setdefault("attn_out_fwd_res_drop", []).append(
            timeit(lambda: ext.gemm_nt_res(x, Wo, b2, dy, 0.1, 1, 2)))
    y = ext.gemm_nt(x, Wo, b2, 0)[0]
    h = ext.gemm_nt_res(x, Wo, b2, dy, 0.1, 1, 2)
    out, hs, mean, rstd = ext.add_ln_fwd(y, dy, g, be, 0.1, 1e-12, 1, 2)
    dout = torch.randn(T, H, device=dev).bfloat16()
    for rep in range(2):
        res.setdefault("ln_fwd_y_res_drop_hcopy", []).append(
            timeit(lambda: ext.add_ln_fwd(y, dy, g, be, 0.1, 1e-12, 1, 2)))
        res.setdefault("ln_fwd_h_only", []).append(
            timeit(lambda: ext.add_ln_fwd(h, None, g, be, 0.0, 1e-12, 0, 0, save_h=False)))
        res.setdefault("ln_bwd_philox", []).append(
            timeit(lambda: ext.add_ln_bwd(dout, hs, mean, rstd, g, 0.1, 1, 2, True, True, True)))
        res.setdefault("ln_bwd_pairhash", []).append(
            timeit(lambda: ext.add_ln_bwd(dout, hs, mean, rstd, g, 0.1, 1, 2, True, True, True, pair_hash=True)))
        res.setdefault("ln_bwd_nodrop", []).append(
            timeit(lambda: ext.add_ln_bwd(dout, hs, mean, rstd, g, 0.0, 1, 2, True, True, True)))
    print(json.dumps({k: [round(v, 4) for v in vs] for k, vs in res.items()}, indent=1))


if __name__ == "__main__":
    main()
