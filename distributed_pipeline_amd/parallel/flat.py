"""
Flat parameter space: every parameter of a module re-homed into ONE contiguous
fp32 master buffer, with its ``.grad`` a view into ONE fp32 gradient buffer
and (for bf16 compute) a view into ONE bf16 shadow buffer.

Why: the reference (utils/trainer.py:91-99, 203-207, 237-271, 360-370) walks
209 tensors for zero_grad, grad norm, AdamW and 3 EMA rates every step.  With a
flat layout each of those is a single memory pass (one kernel), the DDP buckets
are plain slices (no pack/unpack copies, SURVEY K-3), and broadcast at startup
is one collective (SURVEY X-3/X-4).

Layout: parameters are laid out in the order backward completes their gradients -
the module's ``grad_ready_order()`` when it has one, else the *reverse* registration
order - so the gradients produced first (last layers) sit at the front and the
all-reduce buckets fill in order.  Every parameter starts on a 16-element
(64-byte) boundary so views are aligned for 16-byte vector loads; the total is
padded to a multiple of 64 elements.
"""
import math

import torch

ALIGN = 16


def _round_up(x, a):
    return (x + a - 1) // a * a


def unique_trainable(params):
    """Trainable parameters without duplicates (a tied weight appears once), in order."""
    seen, uniq = set(), []
    for p in params:
        if id(p) not in seen and p.requires_grad:
            seen.add(id(p))
            uniq.append(p)
    return uniq


def layout_order(params, reverse=True, order=None):
    """The order :class:`FlatParamSpace` lays ``params`` out in: ``order`` (a module's
    ``grad_ready_order()``: the parameters in the order their gradients complete in the backward)
    when given, else the reverse of the registration order."""
    uniq = unique_trainable(params)
    if order is not None:
        ids = {id(p) for p in uniq}
        lay = [p for p in unique_trainable(order) if id(p) in ids]
        if len(lay) != len(uniq):
            raise ValueError(f"grad_ready_order covers {len(lay)} of {len(uniq)} trainable parameters")
        return lay
    return list(reversed(uniq)) if reverse else uniq


class FlatParamSpace:
    """``break_after`` (layout indices) + ``break_align``: after each of those
    parameters the next offset is rounded up to a multiple of ``break_align``
    elements, so the sharded engine (ZeRO-1, parallel/zero.py) can cut every
    gradient bucket into world-size equal, aligned chunks."""

    def __init__(self, params, device=None, shadow_dtype=None, reverse=True, break_after=(),
                 break_align=ALIGN, order=None):
        uniq = unique_trainable(params)
        self.params = uniq                       # model.parameters() order
        self.layout = layout_order(uniq, reverse, order)
        device = torch.device(device) if device is not None else uniq[0].device
        self.device = device
        self.offsets = {}
        breaks = set(break_after)
        off = 0
        for i, p in enumerate(self.layout):
            self.offsets[id(p)] = off
            off = _round_up(off + p.numel(), ALIGN)
            if i in breaks:
                off = _round_up(off, break_align)
        self.numel = _round_up(max(off, ALIGN), math.lcm(64, break_align))
        self.param_flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad_flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.shadow_flat = (torch.zeros(self.numel, dtype=shadow_dtype, device=device)
                            if shadow_dtype is not None and shadow_dtype != torch.float32 else None)
        # bumped whenever the shadow is rewritten (optimizer step, refresh, ZeRO gather): derived
        # copies of it (the transposed weight shadows of ops/nn.py shadow_t) rebuild once per version
        self.shadow_version = 0
        with torch.no_grad():
            for p in self.layout:
                o, n = self.offsets[id(p)], p.numel()
                self.param_flat[o:o + n].copy_(p.detach().reshape(-1).to(torch.float32))
                p.data = self.param_flat[o:o + n].view(p.shape)
                if p.grad is not None:  # keep already-accumulated gradients
                    self.grad_flat[o:o + n].copy_(p.grad.detach().reshape(-1))
                p.grad = self.grad_flat[o:o + n].view(p.shape)
                if self.shadow_flat is not None:
                    p._dpa_shadow = self.shadow_flat[o:o + n].view(p.shape)
                    p._dpa_shadow._dpa_space = self
        self.refresh_shadow()

    # -- views ---------------------------------------------------------------
    def view(self, flat, p):
        o = self.offsets[id(p)]
        return flat[o:o + p.numel()].view(p.shape)

    def views(self, flat):
        """Per-parameter views of ``flat`` in model.parameters() order."""
        return [self.view(flat, p) for p in self.params]

    def range_of(self, p):
        o = self.offsets[id(p)]
        return o, o + p.numel()

    # -- maintenance -----------------------------------------------------------
    def refresh_shadow(self):
        if self.shadow_flat is not None:
            from ..ops.optim import cast_bf16_
            cast_bf16_(self.param_flat, self.shadow_flat)
            self.shadow_version += 1

    def shadow_written(self):
        """The shadow was rewritten in place (fused optimizer, all-gather)."""
        self.shadow_version += 1

    def zero_grad(self):
        self.grad_flat.zero_()

    def reattach_grads(self):
        """Re-point ``.grad`` at the flat buffer (if user code replaced it)."""
        for p in self.layout:
            g = p.grad
            v = self.view(self.grad_flat, p)
            if g is None or g.data_ptr() != v.data_ptr():
                if g is not None:
                    v.copy_(g)
                p.grad = v

    def new_like(self, init="zeros"):
        if init == "copy":
            return self.param_flat.clone()
        return torch.zeros_like(self.param_flat)
