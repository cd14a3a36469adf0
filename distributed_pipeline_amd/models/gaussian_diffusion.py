"""
Gaussian diffusion for continuous text embeddings (DiffuSeq, ICLR 2023 -
the workload the reference template is written for; SURVEY Appendix B,
call stack CS-5).

Implements the training objective of DiffuSeq's ``training_losses_seq2seq``:

    x0_mean = Emb(ids);  x0 = x0_mean + sqrt(1 - abar_0) * eps0
    x_t     = sqrt(abar_t) x0 + sqrt(1 - abar_t) eps      (target positions only;
                                                          source positions keep x0)
    x0_hat  = model(x_t, t * 1000 / T)                    (predict_xstart)
    mse     = mean_flat((x0 - x0_hat)^2)   [t == 0: mean_flat((x0_mean - x0_hat)^2)]
    tT      = mean_flat((sqrt(abar_{T-1}) x0)^2)
    decoder_nll = mean_L CE(lm_head(x0), ids)
    loss    = mse + decoder_nll + tT ;   nll = masked CE(lm_head(x0_hat), ids)  (logged)

The CE terms go through the fused linear-cross-entropy op (no [N, V] logits
in memory); ``nll`` is computed without autograd since it is only logged.
"""
import math

import numpy as np
import torch

from ..ops import nn as ops


def betas_for_alpha_bar(num_steps, alpha_bar, max_beta=0.999):
    betas = []
    for i in range(num_steps):
        t1, t2 = i / num_steps, (i + 1) / num_steps
        betas.append(min(1 - alpha_bar(t2) / alpha_bar(t1), max_beta))
    return np.array(betas, dtype=np.float64)


def get_named_beta_schedule(name, num_steps):
    if name == "linear":
        scale = 1000 / num_steps
        return np.linspace(scale * 0.0001, scale * 0.02, num_steps, dtype=np.float64)
    if name == "cosine":
        return betas_for_alpha_bar(num_steps, lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2)
    if name == "sqrt":
        return betas_for_alpha_bar(num_steps, lambda t: 1 - np.sqrt(t + 0.0001))
    if name == "trunc_cos":
        return betas_for_alpha_bar(num_steps, lambda t: np.cos((t + 0.1) / 1.1 * np.pi / 2) ** 2)
    if name == "trunc_lin":
        scale = 1000 / num_steps
        return np.linspace(scale * 0.0001 + 0.01, scale * 0.02 + 0.01, num_steps, dtype=np.float64)
    if name == "pw_lin":
        scale = 1000 / num_steps
        b0 = np.linspace(scale * 0.0001 + 0.01, 0.1, 10, dtype=np.float64)
        b1 = np.linspace(0.1, scale * 0.02, num_steps - 10, dtype=np.float64)
        return np.concatenate([b0, b1])
    raise NotImplementedError(f"unknown beta schedule: {name}")


def mean_flat(x):
    return x.mean(dim=list(range(1, x.dim())))


class GaussianDiffusion:
    """Noise schedule tables (kept on device) + the seq2seq training loss."""

    def __init__(self, betas, predict_xstart=True, rescale_timesteps=True, learn_sigma=False,
                 sigma_small=False, rescale_learned_sigmas=False):
        if learn_sigma:
            raise NotImplementedError("learn_sigma=True is not supported (DiffuSeq default is False)")
        if rescale_learned_sigmas:
            # guided-diffusion's RESCALED_MSE only rescales the learned-variance (vb) term
            raise ValueError("rescale_learned_sigmas=True needs learn_sigma=True (unsupported)")
        # reverse-process variance of p_sample (DiffuSeq: FIXED_SMALL if sigma_small
        # else FIXED_LARGE); training losses do not depend on it
        self.model_var_type = "fixed_small" if sigma_small else "fixed_large"
        self.predict_xstart = predict_xstart
        self.rescale_timesteps = rescale_timesteps
        betas = np.asarray(betas, dtype=np.float64)
        self.num_timesteps = int(betas.shape[0])
        alphas = 1.0 - betas
        self.betas = betas
        self.alphas_cumprod = np.cumprod(alphas, axis=0)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.sqrt_alphas_cumprod = np.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - self.alphas_cumprod)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = np.log(np.append(self.posterior_variance[1],
                                                               self.posterior_variance[1:]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = ((1.0 - self.alphas_cumprod_prev) * np.sqrt(alphas)
                                     / (1.0 - self.alphas_cumprod))
        # FIXED_LARGE uses betas (with the posterior variance at t = 0)
        self.large_log_variance = np.log(np.append(self.posterior_variance[1], betas[1:]))
        self._dev_tables = {}

    # -- device tables ------------------------------------------------------
    def _table(self, name, device):
        key = (name, str(device))
        t = self._dev_tables.get(key)
        if t is None:
            t = torch.as_tensor(getattr(self, name), dtype=torch.float32, device=device)
            self._dev_tables[key] = t
        return t

    def _extract(self, name, t, ndim):
        v = self._table(name, t.device)[t]
        return v.view(-1, *([1] * (ndim - 1)))

    def scale_timesteps(self, t):
        if self.rescale_timesteps:
            return t.float() * (1000.0 / self.num_timesteps)
        return t

    # -- forward process ----------------------------------------------------
    def q_sample(self, x_start, t, noise, mask=None):
        x_t = (self._extract("sqrt_alphas_cumprod", t, x_start.dim()) * x_start
               + self._extract("sqrt_one_minus_alphas_cumprod", t, x_start.dim()) * noise)
        if mask is None:
            return x_t
        return torch.where(mask.unsqueeze(-1) == 0, x_start, x_t)

    # -- reverse process (sampling; DiffuSeq p_sample / p_sample_loop) -------
    def q_posterior_mean(self, x_start, x_t, t):
        return (self._extract("posterior_mean_coef1", t, x_t.dim()) * x_start
                + self._extract("posterior_mean_coef2", t, x_t.dim()) * x_t)

    @torch.no_grad()
    def p_mean_variance(self, model, x, t, clip_denoised=False, denoised_fn=None):
        """(mean, log variance, predicted x_0) of p(x_{t-1} | x_t) for an x_0-predicting model."""
        out = model(x, self.scale_timesteps(t)).float()
        if not self.predict_xstart:
            raise NotImplementedError("p_mean_variance: eps-prediction models are not supported")
        pred_x0 = out
        if denoised_fn is not None:
            pred_x0 = denoised_fn(pred_x0, t)
        if clip_denoised:
            pred_x0 = pred_x0.clamp(-1, 1)
        name = "posterior_log_variance_clipped" if self.model_var_type == "fixed_small" else "large_log_variance"
        return self.q_posterior_mean(pred_x0, x, t), self._extract(name, t, x.dim()), pred_x0

    @torch.no_grad()
    def p_sample(self, model, x, t, mask=None, x_start=None, clip_denoised=False, denoised_fn=None):
        """One ancestral step x_t -> x_{t-1}; positions with mask == 0 (the source
        sequence) are kept at x_start (DiffuSeq partial noising)."""
        mean, logvar, pred_x0 = self.p_mean_variance(model, x, t, clip_denoised, denoised_fn)
        noise = torch.randn_like(x)
        nonzero = (t != 0).float().view(-1, *([1] * (x.dim() - 1)))
        sample = mean + nonzero * torch.exp(0.5 * logvar) * noise
        if mask is not None and x_start is not None:
            sample = torch.where(mask.unsqueeze(-1) == 0, x_start, sample)
        return sample, pred_x0

    @torch.no_grad()
    def p_sample_loop(self, model, shape, noise=None, mask=None, x_start=None, clip_denoised=False,
                      denoised_fn=None, device=None):
        """Sample x_0 from T steps of the reverse process (returns the final sample)."""
        x = torch.randn(*shape, device=device) if noise is None else noise
        if mask is not None and x_start is not None:
            x = torch.where(mask.unsqueeze(-1) == 0, x_start, x)
        for i in reversed(range(self.num_timesteps)):
            t = torch.full((shape[0],), i, dtype=torch.long, device=x.device)
            x, _ = self.p_sample(model, x, t, mask, x_start, clip_denoised, denoised_fn)
        return x

    # -- loss ---------------------------------------------------------------
    def training_losses(self, model, *args, **kwargs):
        return self.training_losses_seq2seq(model, *args, **kwargs)

    # Take the fused HIP path (csrc/diffusion.hip) for bf16 models on a GPU; the
    # PyTorch formulas below stay the CPU / fp32 path and the kernels' oracle.
    fused = True

    def _fused_ok(self, net, noise):
        if noise is not None or not GaussianDiffusion.fused:
            return False
        emb = getattr(net, "word_embedding", None)
        if emb is None or getattr(net, "compute_dtype", None) != torch.bfloat16:
            return False
        if getattr(net, "emb_scale_factor", 1.0) != 1.0:
            return False
        from ..ops import diffusion as dops
        return dops.available(emb.weight)

    def _training_losses_fused(self, model, net, t, input_ids, input_mask, compute_nll):
        """Same terms as below; embedding gather + noise + q_sample and the mse/tT
        reductions each run as one kernel (noise drawn in-kernel, never stored)."""
        from ..ops import diffusion as dops
        W = net.word_embedding.weight
        dev = W.device
        x_start, x_start16, x_t = dops.emb_qsample(
            W, input_ids, input_mask, t, self._table("sqrt_alphas_cumprod", dev),
            self._table("sqrt_one_minus_alphas_cumprod", dev),
            float(self.sqrt_one_minus_alphas_cumprod[0]))
        model_out = model(x_t, self.scale_timesteps(t))                       # x0_hat (bf16)
        sa_last = float(self.sqrt_alphas_cumprod[self.num_timesteps - 1])
        mse, tT_loss = dops.diffusion_mse(x_start, model_out, input_ids, t, W, sa_last, t0_via_x_start=True)
        terms = {"mse": mse}
        decoder_nll = self.token_discrete_loss(x_start16, net, input_ids)
        if compute_nll:
            side = _nll_side_stream(dev) if getattr(self, "nll_side_ok", False) else None
            if side is not None and torch.is_grad_enabled():
                # the logged nll needs nothing from the backward and nothing of it needs the
                # nll: it runs on a side stream, joined before the step logs (join_side())
                cur = torch.cuda.current_stream(dev)
                side.wait_stream(cur)
                with torch.cuda.stream(side), torch.no_grad():
                    terms["nll"] = self.token_discrete_loss(model_out.detach(), net, input_ids,
                                                            mask=input_mask)
                for tt in (model_out, input_ids, input_mask, terms["nll"]):
                    tt.record_stream(side)
                self._side_pending = side
            else:
                with torch.no_grad():
                    terms["nll"] = self.token_discrete_loss(model_out.detach(), net, input_ids,
                                                            mask=input_mask)
        terms["decoder_nll"] = decoder_nll
        terms["loss"] = mse + decoder_nll + tT_loss
        return terms

    def join_side(self):
        """Make the current stream wait for a side-stream nll (see _training_losses_fused)."""
        side = getattr(self, "_side_pending", None)
        if side is not None:
            torch.cuda.current_stream(side.device).wait_stream(side)
            self._side_pending = None

    def training_losses_seq2seq(self, model, x_start_unused, t, model_kwargs, noise=None,
                                compute_nll=True):
        """DiffuSeq loss terms, each [B] fp32.  ``model`` may be wrapped (DDP engine)."""
        net = getattr(model, "module", model)
        input_ids = model_kwargs["input_ids"]
        input_mask = model_kwargs["input_mask"]
        if self._fused_ok(net, noise):
            return self._training_losses_fused(model, net, t, input_ids, input_mask, compute_nll)
        x0_mean = net.get_embeds(input_ids)                                  # [B, L, E] fp32
        std0 = float(self.sqrt_one_minus_alphas_cumprod[0])
        x_start = x0_mean + std0 * torch.randn_like(x0_mean)
        if noise is None:
            noise = torch.randn_like(x_start)
        x_t = self.q_sample(x_start, t, noise, mask=input_mask)
        model_out = model(x_t, self.scale_timesteps(t)).float()             # x0_hat
        terms = {}
        mse = mean_flat((x_start - model_out) ** 2)
        t0_loss = mean_flat((x0_mean - model_out) ** 2)
        terms["mse"] = torch.where(t == 0, t0_loss, mse)
        sa_last = float(self.sqrt_alphas_cumprod[self.num_timesteps - 1])
        tT_loss = mean_flat((sa_last * x_start) ** 2)
        decoder_nll = self.token_discrete_loss(x_start, net, input_ids)
        if compute_nll:
            with torch.no_grad():
                terms["nll"] = self.token_discrete_loss(model_out.detach(), net, input_ids,
                                                        mask=input_mask)
        terms["decoder_nll"] = decoder_nll
        terms["loss"] = terms["mse"] + decoder_nll + tT_loss
        return terms

    @staticmethod
    def token_discrete_loss(x, net, input_ids, mask=None):
        """Per-sample CE of the rounding head (DiffuSeq ``_token_discrete_loss``)."""
        B, L = input_ids.shape
        if mask is not None and not torch.is_grad_enabled() and x.is_cuda:
            # only masked tokens count (the logged nll): sort them first and mark the rest
            # ignored, so the fused CE kernel skips whole blocks of them (same values)
            fm = mask.reshape(-1)
            order = _mask_first_order(fm)
            ids_s = torch.where(fm[order] != 0, input_ids.reshape(-1)[order], -100)
            per_s = net.token_nll(x.reshape(B * L, -1)[order], ids_s)
            per_tok = torch.empty_like(per_s).scatter_(0, order, per_s).view(B, L)
        else:
            per_tok = net.token_nll(x.reshape(B * L, -1), input_ids.reshape(-1)).view(B, L)
        if mask is not None:
            m = mask.to(per_tok.dtype)
            return (per_tok * m).sum(-1) / m.sum(-1).clamp_min(1.0)
        return per_tok.mean(-1)


def _mask_first_order(fm):
    """Indices of the nonzero mask entries, then of the zero ones, each in index order: the
    stable 0/1 partition kernel (csrc/sort.hip, two passes over the mask) on the GPU instead
    of a general stable argsort."""
    from ..ops._ext import get_ext
    ext = get_ext() if fm.is_cuda else None
    if ext is not None and hasattr(ext, "partition01") and fm.dtype == torch.int64:
        return ext.partition01(fm)
    return torch.argsort(fm, descending=True, stable=True)


_NLL_SIDE = {}
# the logged nll on its own stream (an A/B hook; off: with the round-5 stream plan it measured
# 0.15-0.37 ms/step slower than inline, profiles/stream_plan_ab_r5.txt)
NLL_SIDE_STREAM = False


def _nll_side_stream(dev):
    """The side stream of the logged nll, or None (NLL_SIDE_STREAM off, CPU, graph capture).
    Overlapping the backward, the forward-only CE sweep over the vocabulary takes CUs while the
    memory-bound kernels run: 164.9 vs 165.6 ms/step (profiles/nll_side_stream_ab_r4.txt).  Only
    a whole-batch step uses it (the trainer sets ``nll_side_ok``): per 64-sample chunk of the
    reference schedule it cost 8-10% (222 -> 241-246 ms/step)."""
    if (not NLL_SIDE_STREAM or dev.type != "cuda"
            or torch.cuda.is_current_stream_capturing()):  # a captured step logs after replay
        return None
    if dev not in _NLL_SIDE:
        # the stream plan's own queue (a torch pool stream shifted which pool streams - hardware
        # queues - an overlapped schedule run later in the process got: 222 -> 240 ms/step)
        from ..runtime.streams import plan_stream
        _NLL_SIDE[dev] = plan_stream(dev, "nll")
    return _NLL_SIDE[dev]


def create_gaussian_diffusion(steps=2000, noise_schedule="sqrt", predict_xstart=True,
                              rescale_timesteps=True, learn_sigma=False, sigma_small=False,
                              rescale_learned_sigmas=False, **_):
    betas = get_named_beta_schedule(noise_schedule, steps)
    return GaussianDiffusion(betas, predict_xstart=predict_xstart,
                             rescale_timesteps=rescale_timesteps, learn_sigma=learn_sigma,
                             sigma_small=sigma_small, rescale_learned_sigmas=rescale_learned_sigmas)
