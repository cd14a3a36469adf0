"""Does the kind of stream change kernel speed?  A large persistent GEMM and a memory-bound
LayerNorm timed on the null stream, a torch pool stream, a plain stream, a CU-masked stream
(full mask) and a high-priority stream; prints each stream's CU mask as read back."""
import json

import torch

from distributed_pipeline_amd.ops._ext import get_ext


def timeit(fn, s, iters=10):
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(iters):
            fn()
        b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ext = get_ext(required=True)
    x = torch.randn(65536, 768, device="cuda").bfloat16()
    W = (torch.randn(3072, 768, device="cuda") * 0.03).bfloat16()
    b = torch.randn(3072, device="cuda").bfloat16()
    g = torch.ones(768, device="cuda").bfloat16()
    be = torch.zeros(768, device="cuda").bfloat16()
    y = torch.randn(262144, 768, device="cuda").bfloat16()
    least, greatest = torch.cuda.Stream.priority_range()
    streams = {"null": torch.cuda.current_stream(), "pool": torch.cuda.Stream(),
               "plain": torch.cuda.ExternalStream(ext.stream_create(0, 0)),
               "cumask": torch.cuda.ExternalStream(ext.stream_create(1, 0)),
               "high": torch.cuda.ExternalStream(ext.stream_create(2, greatest))}
    out = {}
    for name, s in streams.items():
        mask = ext.stream_cu_mask(s.cuda_stream) if s.cuda_stream else None
        out[name] = {"gemm_ms": round(timeit(lambda: ext.gemm_nt(x, W, b, 1), s), 4),
                     "ln_ms": round(timeit(lambda: ext.add_ln_fwd(y, None, g, be, 0.0, 1e-12, 0, 0, save_h=False), s), 4),
                     "cu_mask_bits": None if mask is None else sum(bin(m & 0xffffffff).count("1") for m in mask)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
