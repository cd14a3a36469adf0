"""
ZeRO stage 1 for the native engine (SURVEY §2.2 P-ZeRO: the sharded-optimizer
hook the reference leaves open at utils/trainer.py:246-250, ``opt.clip_grad_norm``).

The AdamW moments and every EMA buffer are partitioned over the data-parallel
group, so a rank keeps (8 + 4 R) / W bytes of optimizer state per parameter
instead of 8 + 4 R (DiffuSeq-XL, 1.32 B parameters, R = 3 EMA rates, W = 8:
26 GB -> 3.3 GB per GPU).  One step:

* backward: the engine REDUCE-SCATTERS each gradient bucket as soon as it is
  complete (``DDPEngine(shard_optimizer=True)``): bucket b is padded to a
  multiple of W x 16 elements and rank r receives the sum of its r-th chunk in
  a compact ``grad_shard`` buffer - no full-size reduced gradient exists;
* grad norm: sum of squares of the local shard + one 1-float all-reduce;
* optimizer: the fused AdamW + EMA kernel (csrc/optim.hip) runs once per bucket
  chunk, on the rank's slice of the fp32 master buffer and its compact m / v /
  EMA shards;
* all-gather: the kernel also writes the updated chunk's bf16 compute shadow, and every
  bucket's shadow chunk is all-gathered (async, half the bytes of fp32); the fp32 master
  outside this rank's chunks is gathered only when needed (``materialize_master``:
  checkpoints, replica checks).

Wire traffic equals DDP's (reduce-scatter + all-gather = all-reduce).  The
checkpoint layout is unchanged: :meth:`state_dict` gathers the moments into
``torch.optim.AdamW`` format and :meth:`ema_params` gathers an EMA - both are
collectives, called on every rank (as ``TrainLoop.save`` does).
"""
import torch

from ..ops import optim as fused
from .optimizer import FusedAdamW


class ZeroFusedAdamW(FusedAdamW):
    """Drop-in for :class:`FusedAdamW` over a sharded :class:`DDPEngine`."""

    def __init__(self, engine, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 ema_rates=()):
        if not engine.sharded:
            raise ValueError("ZeroFusedAdamW needs DDPEngine(shard_optimizer=True) with world > 1")
        self.engine = engine
        super().__init__(engine.space, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                         ema_rates=ema_rates)
        self._sq = torch.zeros(3, dtype=torch.float32, device=engine.space.device)

    def _init_state(self, ema_rates):
        n = self.engine.grad_shard.numel()
        dev = self.space.device
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.ema_rates = [float(r) for r in ema_rates]
        self.ema_flats = [self._shard_of(self.space.param_flat) for _ in self.ema_rates]

    # -- shard <-> full ---------------------------------------------------------
    def _shard_of(self, full):
        out = torch.empty(self.engine.grad_shard.numel(), dtype=full.dtype, device=full.device)
        for s, c, off in self.engine.shard_chunks:
            out[off:off + c].copy_(full[s:s + c])
        return out

    def _gather(self, shard):
        """Full flat buffer (parameter layout) of a sharded state tensor (collective)."""
        full = torch.zeros_like(self.space.param_flat)
        for s, c, off in self.engine.shard_chunks:
            full[s:s + c].copy_(shard[off:off + c])
        self.engine.all_gather_chunks(full)
        return full

    # -- step -------------------------------------------------------------------
    def compute_grad_norm(self, grad_scale=1.0, max_norm=0.0):
        fused.grad_norm_(self.engine.grad_shard, self._sq, self._partial, 1.0, 0.0)
        sq = self._sq[:1] * self._sq[:1]                       # local sum of squares
        self.engine.all_reduce_sum_(sq)
        norm = sq.sqrt() * grad_scale
        coef = (torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0
                else torch.ones_like(norm))
        self.norm_buf.copy_(torch.cat([norm, coef, norm * coef]))
        return self.norm_buf

    def step(self, grad_scale=1.0, clip=None, update_ema=True, skip=None):
        g = self.param_groups[0]
        self.step_count += 1
        b1, b2 = g["betas"]
        p, gs = self.space.param_flat, self.engine.grad_shard
        for s, c, off in self.engine.shard_chunks:
            sl = slice(off, off + c)
            fused.adamw_ema_(p[s:s + c], gs[sl], self.exp_avg[sl], self.exp_avg_sq[sl],
                             lr=g["lr"], beta1=b1, beta2=b2, eps=g["eps"],
                             weight_decay=g["weight_decay"], step=self.step_count,
                             grad_scale=grad_scale, clip=clip,
                             shadow_bf16=None if self.space.shadow_flat is None else self.space.shadow_flat[s:s + c],
                             emas=[e[sl] for e in self.ema_flats] if update_ema else (),
                             ema_rates=self.ema_rates if update_ema else (), skip=skip)
        if self.space.shadow_flat is not None:
            self.space.shadow_written()
        self.engine.gather_params()

    def zero_grad(self, set_to_none=False):  # noqa: ARG002
        self.space.zero_grad()

    # -- checkpoints (collectives) ------------------------------------------------
    def ema_params(self, i):
        return self.space.views(self._gather(self.ema_flats[i]))

    def load_ema(self, i, tensors=None, broadcast=None):
        full = self.space.new_like("copy")
        if tensors is not None:
            with torch.no_grad():
                for dst, src in zip(self.space.views(full), tensors):
                    dst.copy_(src)
        if broadcast is not None:
            broadcast(full)
        self.ema_flats[i].copy_(self._shard_of(full))

    def state_dict(self):
        m, v = self.exp_avg, self.exp_avg_sq
        self.exp_avg, self.exp_avg_sq = self._gather(m), self._gather(v)
        try:
            return super().state_dict()
        finally:
            self.exp_avg, self.exp_avg_sq = m, v

    def load_state_dict(self, sd):
        m_full, v_full = self.space.new_like(), self.space.new_like()
        m, v = self.exp_avg, self.exp_avg_sq
        self.exp_avg, self.exp_avg_sq = m_full, v_full
        try:
            super().load_state_dict(sd)
        finally:
            self.exp_avg, self.exp_avg_sq = m, v
        m.copy_(self._shard_of(m_full))
        v.copy_(self._shard_of(v_full))
