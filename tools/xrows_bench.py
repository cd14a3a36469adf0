"""Micro-bench of the wide-vocabulary CE row pass (csrc/xent_rows.hip xent_rows_fwd_grad_):
GPT-2 shape, 128 MB logit chunks cycled over 1 GB so the row reads come from HBM.
DPA_XROWS_REG=0 selects the looped kernel, 1 (default) the register-resident one."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pipeline_amd.ops._ext import get_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--V", type=int, default=50257)
ap.add_argument("--rows", type=int, default=1310)
ap.add_argument("--chunks", type=int, default=8)
ap.add_argument("--iters", type=int, default=40)
a = ap.parse_args()
ext = get_ext(required=True)
ld = (a.V + 63) // 64 * 64
bufs = [(torch.randn(a.rows, ld, device="cuda") * 3).bfloat16() for _ in range(a.chunks)]
tgt = torch.randint(0, a.V, (a.rows,), device="cuda")
for i in range(a.chunks):
    ext.xent_rows_fwd_grad_(bufs[i], a.V, tgt)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(a.iters):
    ext.xent_rows_fwd_grad_(bufs[i % a.chunks], a.V, tgt)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
gb = 2 * a.rows * ld * 2 / 1e9
print(f"xent_rows_fwd_grad DPA_XROWS_REG={os.environ.get('DPA_XROWS_REG', '1')} V={a.V} rows={a.rows}: "
      f"{ms * 1e3:.1f} us/chunk, {gb / ms:.2f} TB/s (read + write)")
