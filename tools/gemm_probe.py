"""Probe: hipBLASLt (torch.matmul) bf16 throughput on the DiffuSeq-base GEMM shapes,
plus launch overhead of a tiny kernel.  Prints one JSON line per shape."""
import json
import sys
import time

import torch


def bench(fn, iters=50, warmup=10):
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
    dev = torch.device("cuda")
    print(json.dumps({"device": torch.cuda.get_device_name(0),
                      "props": str(torch.cuda.get_device_properties(0))}))
    tokens = [8192, 32768, 131072]
    shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768), (128, 768)]
    for T in tokens:
        for K, N in shapes:
            a = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            ms = bench(lambda: torch.nn.functional.linear(a, w))
            # weight-grad style: [K,T] x [T,N]
            g = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            ms_w = bench(lambda: g.t() @ a)
            fl = 2 * T * K * N
            print(json.dumps({"T": T, "K": K, "N": N, "fwd_ms": round(ms, 4),
                              "fwd_tflops": round(fl / ms / 1e9, 1),
                              "wgrad_ms": round(ms_w, 4), "wgrad_tflops": round(fl / ms_w / 1e9, 1)}))
            sys.stdout.flush()
    x = torch.zeros(16, device=dev)
    ms = bench(lambda: x.add_(1), iters=1000)
    print(json.dumps({"tiny_kernel_ms": ms}))


if __name__ == "__main__":
    main()
