"""
Fused DiffuSeq diffusion-side ops on the gfx950 kernels of ``csrc/diffusion.hip``
(SURVEY K-M1..K-M4, K-M13; the workload of reference utils/trainer.py:1-4):

* :func:`emb_qsample` - word-embedding gather, x_start noise and masked
  ``q_sample`` in one kernel with the noise drawn in-kernel (counter-based
  Philox), returning ``(x_start fp32, x_start bf16, x_t bf16)``.  Its backward
  scatter-adds every gradient reaching the three outputs into the tied
  embedding's fp32 gradient (one atomic pass).
* :func:`diffusion_mse` - the per-sample ``mse`` (with DiffuSeq's t == 0 branch
  against the un-noised embedding) and ``tT`` terms, one workgroup per sample;
  the backward writes d(model output) in its dtype and d(x_start) in fp32.
* :func:`timestep_embedding` - sinusoidal [cos | sin] embedding straight to bf16.

Only used for HIP tensors of a bf16 model; the PyTorch formulas in
``models/gaussian_diffusion.py`` are the CPU / fp32 path and the numerics oracle
of ``tests/test_diffusion_kernels.py``.
"""
import torch

from ._ext import get_ext
from .nn import RNG


def available(W):
    """True when the fused kernels can serve the embedding table ``W``."""
    if not (W.is_cuda and W.dtype == torch.float32 and W.dim() == 2 and W.shape[1] % 4 == 0):
        return False
    ext = get_ext()
    return ext is not None and hasattr(ext, "emb_qsample_fwd")


def _grad_buffer(p):
    """(fp32 buffer to accumulate p's gradient into, tensor to hand to autograd or None).

    The flat engine preallocates ``p.grad`` (a view of the flat gradient buffer): the
    kernels accumulate into it in place and autograd receives None (its
    AccumulateGrad node - and the engine's readiness hook - still runs)."""
    g = p.grad
    if g is not None and g.dtype == torch.float32 and g.is_contiguous() and g.shape == p.shape:
        return g, None
    g = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
    return g, g


def _c(t):
    return None if t is None else t.contiguous()


def _f(t):
    return None if t is None else t.contiguous().float()


class _EmbQSampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, ids, mask, t, sa, s1a, std0, seed, off):
        ctx.set_materialize_grads(False)
        xs, xs16, xt = get_ext().emb_qsample_fwd(ids, mask, t, W.detach(), sa, s1a, float(std0),
                                                 int(seed), int(off), True)
        ctx.save_for_backward(ids, mask, t, sa)
        ctx.W = W
        return xs, xs16, xt

    @staticmethod
    def backward(ctx, d_xs, d_xs16, d_xt):
        ids, mask, t, sa = ctx.saved_tensors
        ret = None
        if ctx.needs_input_grad[0] and any(g is not None for g in (d_xs, d_xs16, d_xt)):
            buf, ret = _grad_buffer(ctx.W)
            get_ext().emb_qsample_bwd(ids, mask, t, sa, _c(d_xs), _c(d_xs16), _c(d_xt), buf)
        return (ret,) + (None,) * 8


class _DiffLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_start, out, ids, t, W, sa_last, t0_via_x_start):
        ctx.set_materialize_grads(False)
        mse, tT = get_ext().diff_loss_fwd(x_start, out, ids, t, W.detach(), float(sa_last))
        ctx.save_for_backward(x_start, out, ids, t)
        ctx.W, ctx.sa_last, ctx.fold = W, float(sa_last), bool(t0_via_x_start)
        return mse, tT

    @staticmethod
    def backward(ctx, dmse, dtT):
        x_start, out, ids, t = ctx.saved_tensors
        if dmse is None and dtT is None:
            return (None,) * 7
        buf = ret = None
        # t == 0 samples: d x0_mean into the embedding rows.  When x_start = W[ids] + noise
        # (emb_qsample) and both get gradients, that term rides on d_xs into the sorted,
        # deterministic embedding backward; otherwise fp32 atomics into W's gradient here.
        fold = ctx.fold and ctx.needs_input_grad[0] and ctx.needs_input_grad[4]
        if ctx.needs_input_grad[4] and dmse is not None and not fold:
            buf, ret = _grad_buffer(ctx.W)
        d_out, d_xs = get_ext().diff_loss_bwd(x_start, out, ids, t, ctx.W.detach(), _f(dmse), _f(dtT),
                                              ctx.sa_last, ctx.needs_input_grad[1],
                                              ctx.needs_input_grad[0], buf, fold_t0=fold)
        return (d_xs if ctx.needs_input_grad[0] else None,
                d_out if ctx.needs_input_grad[1] else None, None, None, ret, None, None)


def emb_qsample(W, ids, mask, t, sqrt_alphas_cumprod, sqrt_one_minus_alphas_cumprod, std0):
    """-> (x_start fp32, x_start bf16, x_t bf16), each [B, L, E]; fresh noise per call."""
    seed, off = RNG.next()
    return _EmbQSampleFn.apply(W, ids.contiguous(), mask.to(torch.long).contiguous(),
                               t.to(torch.long).contiguous(), sqrt_alphas_cumprod,
                               sqrt_one_minus_alphas_cumprod, float(std0), seed, off)


def diffusion_mse(x_start, out, ids, t, W, sqrt_alpha_bar_last, t0_via_x_start=False):
    """-> (mse [B], tT [B]) fp32 (DiffuSeq ``training_losses_seq2seq`` terms).
    ``t0_via_x_start``: x_start is :func:`emb_qsample`'s (W[ids] + noise), so the t == 0 samples'
    embedding gradient may be routed through d x_start (deterministic)."""
    return _DiffLossFn.apply(x_start, out.contiguous(), ids.contiguous(), t.to(torch.long).contiguous(),
                             W, float(sqrt_alpha_bar_last), bool(t0_via_x_start))


def timestep_embedding(timesteps, dim, max_period=10000):
    """Sinusoidal [cos | sin] timestep embedding [B, dim] in bf16."""
    return get_ext().timestep_emb(timesteps.float().contiguous(), int(dim), float(max_period))
