"""
Fused AdamW + multi-rate EMA over a :class:`FlatParamSpace` (SURVEY K-4..K-7).

Numerically the update is ``torch.optim.AdamW`` (decoupled weight decay,
bias-corrected moments); the EMA is the reference's ``update_ema``
(reference: utils/trainer.py:360-370).  One kernel reads g, m, v, p and the R
EMA buffers and writes everything back plus the bf16 compute shadow, with the
DDP 1/world scale and the clip coefficient applied in registers.

``state_dict()``/``load_state_dict()`` produce/consume the exact
``torch.optim.AdamW`` format (per-parameter ``step``/``exp_avg``/
``exp_avg_sq`` keyed by index in ``model.parameters()`` order), so ``opt_*.pt``
checkpoints are interchangeable with the reference's.
"""
import torch

from ..ops import optim as fused


def _torch_adamw_group_defaults():
    p = torch.nn.Parameter(torch.zeros(1))
    g = torch.optim.AdamW([p]).state_dict()["param_groups"][0]
    g.pop("params")
    return g


class FusedAdamW:
    def __init__(self, space, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 ema_rates=()):
        self.space = space
        group = _torch_adamw_group_defaults()
        group.update(lr=float(lr), betas=tuple(betas), eps=float(eps),
                     weight_decay=float(weight_decay))
        group["params"] = list(space.params)
        self.param_groups = [group]
        self.step_count = 0
        self._partial = torch.empty(2048, dtype=torch.float32, device=space.device)
        self.norm_buf = torch.zeros(3, dtype=torch.float32, device=space.device)
        self._init_state(ema_rates)

    def _init_state(self, ema_rates):
        """Moments and EMA buffers (full flat buffers; the ZeRO subclass shards them)."""
        self.exp_avg = self.space.new_like()
        self.exp_avg_sq = self.space.new_like()
        self.ema_rates = [float(r) for r in ema_rates]
        self.ema_flats = [self.space.new_like("copy") for _ in self.ema_rates]

    # -- EMA views (list of per-parameter tensors, model.parameters() order) ----
    def ema_params(self, i):
        return self.space.views(self.ema_flats[i])

    # -- step ---------------------------------------------------------------------
    def compute_grad_norm(self, grad_scale=1.0, max_norm=0.0):
        """Device tensor [norm, clip_coef, norm_after_clip]; no host sync."""
        fused.grad_norm_(self.space.grad_flat, self.norm_buf, self._partial, grad_scale, max_norm)
        return self.norm_buf

    def step(self, grad_scale=1.0, clip=None, update_ema=True, skip=None):
        g = self.param_groups[0]
        self.step_count += 1
        b1, b2 = g["betas"]
        fused.adamw_ema_(self.space.param_flat, self.space.grad_flat, self.exp_avg, self.exp_avg_sq,
                         lr=g["lr"], beta1=b1, beta2=b2, eps=g["eps"], weight_decay=g["weight_decay"],
                         step=self.step_count, grad_scale=grad_scale, clip=clip,
                         shadow_bf16=self.space.shadow_flat,
                         emas=self.ema_flats if update_ema else (),
                         ema_rates=self.ema_rates if update_ema else (), skip=skip)
        if self.space.shadow_flat is not None:
            self.space.shadow_written()

    def zero_grad(self, set_to_none=False):  # noqa: ARG002
        self.space.zero_grad()

    def load_ema(self, i, tensors=None, broadcast=None):
        """Set EMA ``i`` from per-parameter tensors (model.parameters() order, e.g. a
        loaded ``ema_*.pt``; None keeps the current values), then ``broadcast`` the flat
        buffer from rank 0 when given."""
        if tensors is not None:
            with torch.no_grad():
                for dst, src in zip(self.ema_params(i), tensors):
                    dst.copy_(src)
        if broadcast is not None:
            broadcast(self.ema_flats[i])

    # -- torch.optim.AdamW-compatible state ------------------------------------------
    def state_dict(self):
        state = {}
        if self.step_count > 0:
            m = self.space.views(self.exp_avg)
            v = self.space.views(self.exp_avg_sq)
            for i in range(len(self.space.params)):
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": m[i].clone(), "exp_avg_sq": v[i].clone()}
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(g["params"])))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        assert len(groups) == 1, "FusedAdamW holds a single parameter group"
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = tuple(v) if k == "betas" else v
        st = sd.get("state", {})
        m = self.space.views(self.exp_avg)
        v = self.space.views(self.exp_avg_sq)
        steps = set()
        with torch.no_grad():
            for i in range(len(self.space.params)):
                s = st.get(i, st.get(str(i)))
                if s is None:
                    continue
                m[i].copy_(s["exp_avg"])
                v[i].copy_(s["exp_avg_sq"])
                steps.add(int(float(s["step"])))
        if steps:
            self.step_count = max(steps)
