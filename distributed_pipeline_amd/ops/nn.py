"""
Functional compute ops used by the models, with autograd.

Every op here has two implementations:

* the **gfx950 path** (HIP kernels from ``csrc/``), taken for bf16 tensors on a
  HIP device; the kernels are required there (``_ext.get_ext`` raises when the
  extension is missing, so a GPU run can never silently fall back), and
* a **PyTorch reference path** used on CPU and for fp32 (the reference-
  equivalent configuration); it is also the numerics oracle in the tests.

Weights are fp32 ``nn.Parameter``s (views into the engine's flat master
buffer).  For bf16 compute an op reads the parameter's bf16 *shadow*
(``param._dpa_shadow``, refreshed by the fused optimizer) instead of casting
every forward, and returns fp32 weight gradients so they accumulate straight
into the flat fp32 gradient buffer.
"""
import contextlib
import math
import os

import torch
import torch.nn.functional as F

from ._ext import get_ext

# --------------------------------------------------------------------------- #
# helpers
# --------------------------------------------------------------------------- #


def native_ok(*ts, kernel=None):
    """Take the HIP path: all tensors on a HIP device and (if named) the kernel is built."""
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            return False
    ext = get_ext()
    return ext is not None and (kernel is None or hasattr(ext, kernel))


def shadow(p, dtype):
    """Compute-dtype view of parameter ``p`` (bf16 shadow if attached & fresh)."""
    if p is None:
        return None
    if p.dtype == dtype:
        return p
    s = getattr(p, "_dpa_shadow", None)
    if s is not None and s.dtype == dtype:
        return s
    return p.detach().to(dtype)


# Transposed bf16 weight shadows for the data-gradient GEMMs (DPA_WT_SHADOW=0: off): dx = dy W reads
# W^T [K][N] through the forward kernel's row-form operand path instead of W through transposed
# LDS reads, 3-5% faster per call (tools/probes/dgrad_layout.py) for one transpose copy per weight
# and optimizer step.
_WT_SHADOW = os.environ.get("DPA_WT_SHADOW", "1") != "0"


def shadow_t(w16):
    """W^T of a bf16 weight shadow (``param._dpa_shadow``, parallel/flat.py), rebuilt on the current
    stream the first time it is needed after each rewrite of the shadow; None for anything else."""
    if not _WT_SHADOW or w16 is None or w16.dim() != 2:
        return None
    # only shapes the persistent row-form dgrad can tile (dx[T][K] = dy[T][N] . W[N][K]: K % 256,
    # N % 128; launch_gemmp_nn) get a shadow, so no other weight is copied or pinned
    if w16.shape[1] % 256 or w16.shape[0] % 128:
        return None
    sp = getattr(w16, "_dpa_space", None)
    if sp is None or not w16.is_cuda:
        return None
    st = getattr(w16, "_dpa_t", None)
    if st is None:
        st = torch.empty((w16.shape[1], w16.shape[0]), dtype=w16.dtype, device=w16.device)
        w16._dpa_t = st
        w16._dpa_tver = -1
        lst = getattr(sp, "_wt_list", None)
        if lst is None:
            lst = sp._wt_list = []
        lst.append(w16)
    if w16._dpa_tver != sp.shadow_version:
        _refresh_wt(sp)
    WT_STATS["used"] += 1
    return st


def _refresh_wt(sp):
    """Every stale W^T of the space in one batched transpose launch (torch's strided copy per
    weight cost 0.7 ms/step), on the current stream."""
    ver = sp.shadow_version
    stale = [w for w in sp._wt_list if w._dpa_tver != ver]
    ext = get_ext()
    if not (hasattr(ext, "transpose_bf16_batch") and ext.transpose_bf16_batch(stale, [w._dpa_t for w in stale])):
        for w in stale:
            w._dpa_t.copy_(w.t())
    for w in stale:
        w._dpa_tver = ver
    WT_STATS["copies"] += len(stale)
    if _WT_CHECK:  # DPA_DEFER_CHECK=1: every refreshed W^T against the shadow it was built from
        for w in stale:
            if not torch.equal(w._dpa_t, w.t()):
                raise RuntimeError(f"stale or corrupt W^T shadow of a {tuple(w.shape)} weight")


_WT_CHECK = os.environ.get("DPA_DEFER_CHECK", "0") == "1"


WT_STATS = {"used": 0, "copies": 0}


def _mm_fp32(a, b):
    """a @ b with fp32 output (bf16 inputs on GPU keep fp32 accumulation)."""
    if a.is_cuda and a.dtype == torch.bfloat16:
        return torch.mm(a, b, out_dtype=torch.float32)
    return (a.float() @ b.float())


# --------------------------------------------------------------------------- #
# Linear (+ optional fused activation)
# --------------------------------------------------------------------------- #

# index = kernel act code; "deriv" (4): the saved operand is already act'(z); "deriv8" (5):
# act'(z) as u8 codes in the persistent GEMM's tile-native layout (see act_q8_decode)
_ACTS = ("none", "gelu", "tanh", "silu", "deriv", "deriv8")


def act_q8_decode(z8, T, N):
    """[T, N] fp32 act' from the u8 codes of ``gemm_nt(want_deriv=2)``.

    Layout (csrc/gemm256.hip ``q8_off``): byte (((((mt*NT + nt)*8 + w)*8 + ro)*2 + k)*512 + ln*8 + e
    holds element (mt*256 + qa*128 + wm*64 + i*16 + k*8 + ln//8, nt*256 + wn*64 + (ln%8)*8 + e)
    with w = 4 wm + wn and ro = 4 qa + i.  Codes (``q8_code``): min((c - 19) * 0.5 / 74,
    (c + 35) / 256) - the first line below code 93, the second above."""
    c = z8.view(T // 256, N // 256, 2, 4, 2, 4, 2, 8, 8, 8)  # mt nt wm wn qa i k lr lc e
    c = c.permute(0, 4, 2, 5, 6, 7, 1, 3, 8, 9).reshape(T, N).float()
    lo = (c - 19.0) * torch.tensor(0.5 / 74.0, dtype=torch.float32)
    hi = c * (1.0 / 256.0) + 35.0 / 256.0
    return torch.minimum(lo, hi)


def _act_fwd(z, act):
    if act == "none":
        return z
    if act == "gelu":
        return F.gelu(z)
    if act == "tanh":
        return torch.tanh(z)
    if act == "silu":
        return F.silu(z)
    raise ValueError(act)


def _act_bwd(dy, z, y, act):
    """d act(z) given dy, pre-activation z and output y (fp32 math)."""
    if act == "none":
        return dy
    dyf = dy.float()
    if act == "deriv":  # z holds act'(pre-activation), saved by the forward epilogue
        return (dyf * z.float()).to(dy.dtype)
    if act == "deriv8":  # the same as u8 codes
        return (dyf * act_q8_decode(z, dy.shape[0], dy.shape[1])).to(dy.dtype)
    if act == "tanh":
        yf = y.float()
        return (dyf * (1.0 - yf * yf)).to(dy.dtype)
    zf = z.float()
    if act == "gelu":
        cdf = 0.5 * (1.0 + torch.erf(zf * (1.0 / math.sqrt(2.0))))
        pdf = torch.exp(-0.5 * zf * zf) * (1.0 / math.sqrt(2.0 * math.pi))
        return (dyf * (cdf + zf * pdf)).to(dy.dtype)
    if act == "silu":
        s = torch.sigmoid(zf)
        return (dyf * (s * (1.0 + zf * (1.0 - s)))).to(dy.dtype)
    raise ValueError(act)


def _bias_act_fwd(z2d, b16, act):
    if native_ok(z2d, kernel="bias_act_fwd") and z2d.dtype == torch.bfloat16 and z2d.shape[-1] % 8 == 0:
        return get_ext().bias_act_fwd(z2d, b16, _ACTS.index(act))
    z = z2d if b16 is None else z2d + b16
    return z, _act_fwd(z, act)


def _bias_act_bwd(dy2d, z, y, act, want_db):
    if act == "deriv8":
        z, act = act_q8_decode(z, dy2d.shape[0], dy2d.shape[1]).to(dy2d.dtype), "deriv"
    if native_ok(dy2d, kernel="bias_act_bwd") and dy2d.dtype == torch.bfloat16 and dy2d.shape[-1] % 8 == 0:
        zy = z if z is not None else (y if y is not None else dy2d)
        dz, db = get_ext().bias_act_bwd(dy2d, zy, _ACTS.index(act), want_db)
        return dz, (db if want_db else None)
    dz = _act_bwd(dy2d, z, y, act)
    db = dz.float().sum(0) if want_db else None
    return dz, db


# Linear GEMM routing (GEMM_MODE):
#   "auto" / "native" (default) - every Linear GEMM on the hand-written gfx950
#            kernels: forward and data-gradient GEMMs on the persistent 256 x 256
#            kernel of csrc/gemm256.hip (bias, activation and pre-activation copy
#            fused into the forward epilogue; the previous layer's activation
#            backward and its bias gradient fused into the data-gradient epilogue),
#            weight gradients on the split-K kernel that accumulates into the fp32
#            grad buffer.  Measured against hipBLASLt + separate elementwise passes
#            at 262144 tokens: profiles/gemm_lab_r2.txt;
#   "blas"   - every Linear GEMM on hipBLASLt (plus separate epilogue kernels), the
#            A/B reference.
GEMM_MODE = "auto"  # "blas": stock torch.mm for every Linear (tests / A/B; set the attribute)
# post-LN attention sublayer at L = 128: QKV stored head-major for the attention kernels
_QKV_HEAD_MAJOR = True
# forward GEMM epilogues store act'(z) instead of z for the backward (DPA_SAVE_ACT_DERIV=0: z)
_SAVE_ACT_DERIV = os.environ.get("DPA_SAVE_ACT_DERIV", "1") != "0"
# ... and, for the fused MLP (whose backward is the persistent dact GEMM), as 8-bit codes:
# half the bytes of the largest store / load pair of the step (DPA_ACT_Q8=0: bf16 act')
_ACT_Q8 = os.environ.get("DPA_ACT_Q8", "1") != "0"
# post-LN sublayers: residual + dropout of the branch output in the producing GEMM's epilogue
# (h = x + dropout(y) written once; the LayerNorm reads h alone and writes no h copy)
# (DPA_RES_FUSE=0: the GEMM writes y and the LayerNorm kernel adds the residual)
_RES_FUSE = os.environ.get("DPA_RES_FUSE", "1") != "0"
# post-LN sublayers keep the exact h copy for the LayerNorm backward.  (An output-based backward
# reconstructing xhat from the sublayer's output measured 1.9-2.0 ms/step slower in round 4,
# profiles/ln_save_out_ab_r4.txt, and was retired in round 6; the kernel's h_guard mode stays
# for the norm tests.)


def _gemm_shape_ok(x2, n_out):
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and native_ok(x2, kernel="gemm_nt")
            and x2.shape[0] % 128 == 0 and n_out % 128 == 0 and x2.shape[1] % 128 == 0)


# Small token counts (the time-embedding MLP runs on [B, 128] rows: B = 64 in the reference
# 32 x 64 schedule) are padded with zero rows to a multiple of 128 so the native MFMA GEMMs
# take them instead of hipBLASLt.  Zero rows add nothing to the weight / bias gradients
# (their output gradient is zero) and are sliced off the outputs and the input gradient.
_PAD_ROWS = 128
_PAD_MAX_T = 8192
PAD_STATS = {"padded": 0}


def _pad_rows(x2, n_outs):
    """x2 zero-padded to a multiple of 128 rows when that makes the native GEMMs eligible
    (else x2 itself), and the original row count."""
    T = x2.shape[0]
    if (T % _PAD_ROWS == 0 or T > _PAD_MAX_T or GEMM_MODE == "blas" or not x2.is_cuda
            or x2.dtype != torch.bfloat16 or x2.shape[1] % 128 or any(n % 128 for n in n_outs)
            or not native_ok(x2, kernel="gemm_nt")):
        return x2, T
    Tp = -(-T // _PAD_ROWS) * _PAD_ROWS
    PAD_STATS["padded"] += 1
    xp = x2.new_zeros(Tp, x2.shape[1])
    xp[:T].copy_(x2)
    return xp, T


def _pad_grad(dy2, Tp):
    if dy2.shape[0] == Tp:
        return dy2
    dp = dy2.new_zeros(Tp, dy2.shape[1])
    dp[:dy2.shape[0]].copy_(dy2)
    return dp


def _route(x2, n_out, act):
    """-> (native_fwd, native_dgrad, native_wgrad)"""
    if GEMM_MODE == "blas" or not _gemm_shape_ok(x2, n_out):
        return False, False, False
    return True, True, True


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class _WgradDeferral:
    """Weight-gradient deferral for the reference (micro-batch) schedule.

    Under ``no_sync`` the weight gradient of micro-batch k is only needed once the whole
    step's micro-batches have been accumulated (reference: ``loss.backward()`` per micro-batch
    inside ``no_sync``, /root/reference/utils/trainer.py:209-235).  An 8192-token micro-batch
    gives a 768 x 768 weight 9 output tiles, so the split-K GEMM splits the tokens ~14 ways and
    merges 14 fp32 partial slabs per call - more HBM traffic than the GEMM's own operands.
    With ``depth`` = d the (dy, x) operands of a Linear are held for d - 1 micro-batches and
    the d segments run as ONE multi-segment split-K launch (each segment split fewer ways, one
    reduce pass): the same sum into the same fp32 gradient, at most d - 1 micro-batches of
    extra operand memory.  ``active`` is set by the trainer around every backward except the
    last (DDP-armed) one, before which ``flush()`` runs whatever is still held.

    Grouped flushes (``grouped``): the sites that complete their d segments in a backward are not
    launched one by one (a split-K launch each, whose fp32 partial slabs a reduce pass merges) but
    together after it (``end_backward``), as ONE grouped kernel over all their 256 x 256 tiles
    (~1300 for DiffuSeq-base: ~5 rounds of the CUs, so no token split, no slabs, no reduce; each
    dW element has one writer)."""

    def __init__(self):
        self.depth = 0
        self.active = False
        self.pending = {}  # id(weight) -> (weight, bias, [(dz, x2), ...])
        self.held_bytes = 0
        # operands are only held while their total stays under this budget (a large executed
        # micro-batch - DiffuSeq-XL's 1024-sample chunks hold ~100 GB of Linear operands -
        # gains nothing from deferral and must not double its memory)
        self.budget_bytes = int(float(os.environ.get("DPA_DEFER_WGRAD_GB", "32")) * (1 << 30))
        self.stats = {"deferred": 0, "multi_launches": 0, "segments": 0, "ln_deferred": 0, "ln_reduces": 0,
                      "bias_deferred": 0, "bias_reduces": 0, "attn_deferred": 0, "attn_reduces": 0,
                      "group_launches": 0, "group_sites": 0}
        # sites whose segments are complete in the current backward: launched together by
        # end_backward() (or flush()) as ONE grouped weight-gradient kernel
        self.ready = []
        self.stream = None  # side stream for the un-armed micro-batches' launches (trainer-set)
        self.cur = None     # the stream the current backward runs on (trainer-set, optional)
        self._retired = []  # replaced column-sum buffers (other streams may still use them)
        # Column-sum deferral (same window): a LayerNorm backward at 8192 rows writes 1024
        # block partials of its dgamma / dbeta / dy column sums and a second kernel reduces
        # them (~7 us, on the backward chain, 26 per micro-batch); a fused dact GEMM's bias
        # partials likewise.  While deferring, the LN kernel ADDS its partials onto a per-site
        # buffer and the dact GEMM writes into consecutive slots of a per-bias buffer; one
        # reduction per site runs at flush().
        self.ln_sites = {}    # id(gamma) -> [buf, R, D, dg, db, dyb, filled]
        self.bias_sites = {}  # id(bias) -> [buf, rows, K, gb, used]
        # the attention backward's qkv-bias partials likewise ([rows][3 D] per call, ext.attn_bwd
        # part_out): one colpart reduction per site and flush instead of one per micro-batch
        self.attn_sites = {}  # id(bias) -> [buf, rows, H, D, gb, used]
        self.colsum = True
        # debug (DPA_DEFER_CHECK=1): checksum every held operand when it is held and again when
        # its launch runs - a held tensor whose memory was rewritten meanwhile is reported
        self.check = os.environ.get("DPA_DEFER_CHECK", "0") == "1"
        self.check_log = []

    @staticmethod
    def _sig(t):
        return (float(t.detach().float().sum()), float(t.detach().float().abs().sum()))

    def _verify(self, p, segs):
        for i, s in enumerate(segs):
            if len(s) > 2:
                now = (self._sig(s[0]), self._sig(s[1]))
                if now != s[2]:
                    self.check_log.append((tuple(p.shape), i, s[2], now))

    def _cur(self, t):
        """The current stream (``cur``: set by the trainer per micro-batch, saving the
        device-index lookup of ``torch.cuda.current_stream`` on every offer)."""
        if self.cur is not None:
            return self.cur
        return torch.cuda.current_stream(t.device) if t.is_cuda else None

    # grouped flushes (one kernel over every complete site, csrc/gemm256.hip wgrad_group_kernel);
    # False: one split-K launch per site.  A group runs when its sites have at least
    # group_min_tiles 256 x 256 tiles (None: one per CU; fewer are split-K per site, which fills
    # the chip by splitting the tokens)
    grouped = True
    group_min_tiles = None

    @staticmethod
    def _gb(bias):
        return bias.grad if (bias is not None and bias.requires_grad) else None

    def _stream_for(self, segs, side):
        """(current stream, stream to launch on) - ``side``: ``self.stream``, ordered after the
        current stream's work so far; the held operands are kept alive for it."""
        cur = self._cur(segs[0][0])
        run_on = cur
        if cur is not None and side and self.stream is not None:
            run_on = self.stream
            run_on.wait_stream(cur)
        return cur, run_on

    def _run(self, p, bias, segs, side=False):
        """Launch the held segments.  ``side``: on ``self.stream`` (ordered after the current
        stream's work so far) instead of the current stream - the weight gradients of the
        un-armed micro-batches are off the backward chain's critical path; nothing reads
        them before the trainer joins that stream ahead of the last backward."""
        cur, run_on = self._stream_for(segs, side)
        if self.check:
            self._verify(p, segs)
        segs = [s[:2] for s in segs]
        if run_on is not None:
            for dz, x2 in segs:  # produced on other streams: keep them alive for run_on
                dz.record_stream(run_on)
                x2.record_stream(run_on)
        with torch.cuda.stream(run_on) if run_on is not None and run_on is not cur else _nullctx():
            self._launch_site(p, bias, segs)

    def _launch_site(self, p, bias, segs):
        ext = get_ext()
        gw, gb = p.grad, self._gb(bias)
        if len(segs) > 1 and ext.gemm_wgrad_multi([s[0] for s in segs], [s[1] for s in segs], gw, gb):
            self.stats["multi_launches"] += 1
            self.stats["segments"] += len(segs)
            return
        for dz, x2 in segs:
            ext.gemm_wgrad(dz, x2, gw, gb)

    @staticmethod
    def _groupable(segs):
        dz, x2 = segs[0][0], segs[0][1]
        return (len(segs) <= 8 and dz.shape[1] % 256 == 0 and x2.shape[1] % 256 == 0 and dz.shape[0] % 128 == 0
                and dz.shape[0] >= 128)

    def _run_group(self, items, side=True):
        """Every site of ``items`` ((weight, bias, segs, ...)): the ones that tile as ONE grouped
        launch when together they fill the chip (no token split, no reduce pass), the rest one by
        one."""
        if not items:
            return
        ext = get_ext()
        grp, seen = [], set()
        for it in items:  # one entry per weight: two sites adding into one dW must not share a launch
            if self.grouped and it[2][0][0].is_cuda and self._groupable(it[2]) and id(it[0]) not in seen:
                grp.append(it)
                seen.add(id(it[0]))
        if grp and hasattr(ext, "gemm_wgrad_grouped"):
            tiles = sum((it[2][0][0].shape[1] // 256) * (it[2][0][1].shape[1] // 256) for it in grp)
            dev = grp[0][2][0][0].device
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 1
            if len(grp) > 1 and tiles >= (ncu if self.group_min_tiles is None else self.group_min_tiles):
                cur, run_on = self._stream_for(grp[0][2], side)
                for p, _b, segs, *_ in grp:
                    if self.check:
                        self._verify(p, segs)
                    if run_on is not None:
                        for s in segs:
                            s[0].record_stream(run_on)
                            s[1].record_stream(run_on)
                with torch.cuda.stream(run_on) if run_on is not None and run_on is not cur else _nullctx():
                    ok = ext.gemm_wgrad_grouped([[s[0] for s in it[2]] for it in grp],
                                                [[s[1] for s in it[2]] for it in grp],
                                                [it[0].grad for it in grp], [self._gb(it[1]) for it in grp])
                    if ok:
                        self.stats["group_launches"] += 1
                        self.stats["group_sites"] += len(grp)
                        self.stats["segments"] += sum(len(it[2]) for it in grp)
                    else:
                        for p, b, segs, *_ in grp:
                            self._launch_site(p, b, [s[:2] for s in segs])
                done = {id(it) for it in grp}
                items = [it for it in items if id(it) not in done]
        for p, b, segs, *_ in items:
            self._run(p, b, segs, side=side)

    def end_backward(self):
        """Launch the sites that completed their segments in this backward, grouped."""
        items, self.ready = self.ready, []
        for it in items:
            self.held_bytes -= it[3]
        self._run_group(items, side=True)

    def offer(self, p, dz, x2, bias, gw, gb):
        """True when the weight gradient was deferred or run here (grads preallocated)."""
        if self.depth < 2 or gw is not p.grad or (gb is not None and gb is not bias.grad):
            return False
        key = id(p)
        ent = self.pending.pop(key, None)
        if ent is not None:
            segs, nb = ent[2], ent[3]
            self.held_bytes -= nb
            if (segs[0][0].shape != dz.shape or segs[0][1].shape != x2.shape
                    or (ent[1] is not None) != (bias is not None)):
                self._run(ent[0], ent[1], segs)
                segs, nb = [], 0
        else:
            segs, nb = [], 0
        segs.append((dz, x2, (self._sig(dz), self._sig(x2))) if self.check else (dz, x2))
        nb += dz.numel() * dz.element_size() + x2.numel() * x2.element_size()
        if self.active and len(segs) < self.depth and self.held_bytes + nb <= self.budget_bytes:
            self.pending[key] = (p, bias, segs, nb)
            self.held_bytes += nb
            self.stats["deferred"] += 1
            return True
        if (self.active and self.grouped and len(segs) >= self.depth
                and self.held_bytes + nb <= self.budget_bytes):  # complete: launched with the others by end_backward()
            self.ready.append((p, bias, segs, nb))
            self.held_bytes += nb
            return True
        self._run(p, bias, segs, side=self.active)
        return True

    def flush(self):
        """Run every held weight gradient (on the side stream when set) and every deferred
        column-sum reduction (on the current stream)."""
        pend, self.pending = self.pending, {}
        ready, self.ready = self.ready, []
        self.held_bytes = 0
        self._run_group(ready + list(pend.values()), side=True)
        for e in self.ln_sites.values():
            self._ln_reduce(e)
        for e in self.bias_sites.values():
            self._bias_reduce(e)
        for e in self.attn_sites.values():
            self._attn_reduce(e)

    def release_retired(self, stream):
        """Free the replaced column-sum buffers once ``stream`` has joined every stream that
        could still use them (the trainer calls this after the overlapped schedule's joins):
        ``record_stream`` keeps the allocator from reusing a block before the work queued on
        ``stream`` so far - which follows all of it - has run."""
        for b in self._retired:
            if stream is not None and b.is_cuda:
                b.record_stream(stream)
        self._retired = []

    def drop(self):
        """Forget held operands (an abandoned backward whose gradients are discarded)."""
        self.pending = {}
        self.ready = []
        self.held_bytes = 0
        self.active = False
        for e in self.ln_sites.values():
            e[6] = False
        for e in self.bias_sites.values():
            e[4] = 0
        for e in self.attn_sites.values():
            e[5] = 0

    # ---- column sums -----------------------------------------------------------------
    def _colsum_on(self):
        return self.colsum and self.active and self.depth >= 2

    @staticmethod
    def _same(a, b):
        return (a is None) == (b is None) and (a is None or a.data_ptr() == b.data_ptr())

    def _ln_reduce(self, e):
        if e[6]:
            get_ext().ln_colreduce(e[0], e[1], e[2], e[3], e[4], e[5])
            e[6] = False
            self.stats["ln_reduces"] += 1

    def ln_part(self, gamma, R, D, dg, db, dyb):
        """(partial buffer, accumulate) for a deferred LayerNorm backward of gamma's site, or
        (None, False).  dg / db (/ dyb) must be the .grad buffers the reduction adds onto."""
        if not self._colsum_on() or dg is None or db is None:
            return None, False
        n = get_ext().ln_bwd_partials(R, D)
        if n <= 0:
            return None, False
        e = self.ln_sites.get(id(gamma))
        if e is not None and (e[1] != R or e[2] != D or not self._same(e[3], dg) or not self._same(e[4], db)
                              or not self._same(e[5], dyb)):
            self._ln_reduce(e)
            buf = e[0] if e[0].numel() == n else None
            if buf is None:
                self._retired.append(e[0])
            e = None
        else:
            buf = None if e is None else e[0]
        if e is None:
            if buf is None:
                buf = torch.empty(n, dtype=torch.float32, device=dg.device)
            e = [buf, R, D, dg, db, dyb, False]
            self.ln_sites[id(gamma)] = e
        # the site buffers live as long as this object (replaced ones in _retired): no
        # record_stream needed when the backward alternates streams
        acc = e[6]
        e[6] = True
        self.stats["ln_deferred"] += 1
        return buf, acc

    BIAS_SLOTS = 8

    def _bias_reduce(self, e):
        if e[4]:
            get_ext().colsum_acc(e[0][: e[4] * e[1]], e[3])
            e[4] = 0
            self.stats["bias_reduces"] += 1

    def bias_part(self, bias, gb, T, K):
        """A [(T/256)*2, K] fp32 slot for a fused dact GEMM's bias partials (reduced onto gb
        at flush or when the site's slots are full), or None."""
        if not self._colsum_on() or gb is None or T % 256:
            return None
        rows = (T // 256) * 2
        e = self.bias_sites.get(id(bias))
        if e is not None and (e[1] != rows or e[2] != K or not self._same(e[3], gb)):
            self._bias_reduce(e)
            self._retired.append(e[0])
            e = None
        if e is None:
            e = [torch.empty(self.BIAS_SLOTS * rows, K, dtype=torch.float32, device=gb.device), rows, K, gb, 0]
            self.bias_sites[id(bias)] = e
        if e[4] == self.BIAS_SLOTS:
            self._bias_reduce(e)
        slot = e[0][e[4] * rows:(e[4] + 1) * rows]
        e[4] += 1
        self.stats["bias_deferred"] += 1
        return slot


    ATTN_SLOTS = 8

    def _attn_reduce(self, e):
        if e[5]:
            get_ext().attn_colpart_reduce(e[0], e[5] * e[1] // e[2], e[2], e[3], e[4])
            e[5] = 0
            self.stats["attn_reduces"] += 1

    def attn_part(self, bias, gb, rows, H, D):
        """A [rows * 3 D] fp32 slot for an attention backward's qkv-bias partials (rows =
        ext.attn_colpart_rows), reduced onto gb at flush or when the site's slots are full; or None."""
        if not self._colsum_on() or gb is None or rows % H or not hasattr(get_ext(), "attn_colpart_reduce"):
            return None  # (an extension built before deferred attention partials: A/B variants)
        n = rows * 3 * D
        e = self.attn_sites.get(id(bias))
        if e is not None and (e[1] != rows or e[2] != H or e[3] != D or not self._same(e[4], gb)):
            self._attn_reduce(e)
            self._retired.append(e[0])
            e = None
        if e is None:
            e = [torch.empty(self.ATTN_SLOTS * n, dtype=torch.float32, device=gb.device), rows, H, D, gb, 0]
            self.attn_sites[id(bias)] = e
        if e[5] == self.ATTN_SLOTS:
            self._attn_reduce(e)
        slot = e[0][e[5] * n:(e[5] + 1) * n]
        e[5] += 1
        self.stats["attn_deferred"] += 1
        return slot


WGRAD_DEFER = _WgradDeferral()


def _accumulate_wgrad(p, dz, x2, bias):
    """dW (+db) straight into the parameters' fp32 .grad buffers via the split-K GEMM.

    Returns (dw, db) tensors only when a parameter has no preallocated gradient.
    """
    ext = get_ext()
    dw_out = db_out = None
    gw = p.grad if _INPLACE[0] else None
    if gw is None or gw.dtype != torch.float32 or not gw.is_contiguous():
        gw = dw_out = torch.zeros(p.shape, dtype=torch.float32, device=dz.device)
    gb = None
    if bias is not None and bias.requires_grad:
        gb = bias.grad if _INPLACE[0] else None
        if gb is None or gb.dtype != torch.float32:
            gb = db_out = torch.zeros(bias.shape, dtype=torch.float32, device=dz.device)
    if WGRAD_DEFER.offer(p, dz, x2, bias, gw, gb):
        return None, None
    ext.gemm_wgrad(dz, x2, gw, gb)
    # Readiness needs no explicit signal: autograd still runs the parameter's
    # AccumulateGrad node (with an undefined grad) after this backward, and its
    # post-accumulate hook - the DDP engine's bucket counter - fires exactly once
    # per backward, after every use of the parameter has been processed.
    return dw_out, db_out


def _lin_fwd(x2, w16, b16, act, route, q8=False):
    """Forward GEMM (+bias, +activation) of one Linear -> (y, z, zact).

    z is what the activation backward needs (gelu/silu; tanh's backward uses y):
    on the persistent kernel act'(pre-activation), computed in the forward epilogue
    together with act (the erf/exp work is shared, and the backward epilogue becomes
    one multiply), else the pre-activation.  zact names the backward rule for z:
    "deriv", "deriv8" (q8: u8 codes, only for a backward through gemm_nn_dact) or ``act``."""
    if route[0]:
        want = 0
        if _SAVE_ACT_DERIV and act in ("gelu", "silu"):
            want = 2 if (q8 and _ACT_Q8) else 1
        y, z, mode = get_ext().gemm_nt(x2, w16, b16, _ACTS.index(act), want)
        if act in ("gelu", "silu"):
            return y, z, ("deriv8" if mode == 2 else "deriv" if mode == 1 else act)
    else:
        if b16 is not None and x2.is_cuda:
            z = torch.addmm(b16, x2, w16.t())  # hipBLASLt bias epilogue
            b16_epi = None
        else:
            z = x2 @ w16.t()
            b16_epi = b16
        if b16_epi is not None or act != "none":
            z, y = _bias_act_fwd(z, b16_epi, act)
        else:
            y = z
    return y, (z if act in ("gelu", "silu") else None), act


# Bias-gradient hand-off.  The kernel that produces a Linear's output gradient
# often reads every element of it anyway (LayerNorm backward, attention
# backward, activation backward) and column-sums it for free; it offers the sum
# here and the Linear's backward takes it, so the wgrad GEMM does not reduce dz
# a second time (measured: +30% wgrad time for the in-GEMM column sum).
_DB_OFFER = [None]
DB_HANDOFF_STATS = {"offered": 0, "taken": 0, "fused_sublayers": 0}


def _offer_db(g, db):
    _DB_OFFER[0] = (g, db) if db is not None else None
    DB_HANDOFF_STATS["offered"] += db is not None


def _take_db(g):
    """The offered column sum of ``g`` (same storage, same numel), else None.
    Always clears the slot so an unclaimed offer does not pin its gradient."""
    o, _DB_OFFER[0] = _DB_OFFER[0], None
    if o is None:
        return None
    og, db = o
    if og.data_ptr() == g.data_ptr() and og.numel() == g.numel() and db.numel() == g.shape[-1]:
        DB_HANDOFF_STATS["taken"] += 1
        return db
    return None


# marker for ``_lin_param_grads(..., db=_ACCUMULATED)``: the bias gradient was already
# added onto ``b.grad`` in place by the kernel that produced it
_ACCUMULATED = object()


_GRAD_ACC = True
# In-place parameter gradients are an engine-internal contract: only inside the trainer's own
# backward (``inplace_param_grads``) do the ops add into ``.grad`` and hand None to autograd.
# Anywhere else (a user's ``loss.backward()``, ``torch.autograd.grad`` for a gradient penalty or
# a norm probe) every parameter gradient is returned to autograd as usual.
_INPLACE = [False]


@contextlib.contextmanager
def inplace_param_grads(on=True):
    """Let the ops accumulate parameter gradients straight into the flat fp32 ``.grad`` buffers
    for the duration (utils/trainer.py wraps its backward passes in this)."""
    prev = _INPLACE[0]
    _INPLACE[0] = bool(on)
    try:
        yield
    finally:
        _INPLACE[0] = prev


def _grad_acc(p):
    """``p.grad`` when a kernel can accumulate onto it in place (the flat fp32 gradient
    buffer views of the DDP engine, inside ``inplace_param_grads``), else None (the gradient
    is returned to autograd)."""
    if p is None or not _GRAD_ACC or not _INPLACE[0]:
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g


def _into_grad(p, g):
    """Add a parameter gradient in place into ``p.grad`` when that is a flat fp32 buffer view
    (native DDP engine) and return None to autograd, else return ``g``.  Nothing then reaches
    the parameter's AccumulateGrad node: in the overlapped micro-batch schedule the backwards
    alternate between two HIP streams while each AccumulateGrad node keeps the stream it was
    created on, so a materialised gradient would make autograd order the two streams against
    each other (torch's "AccumulateGrad node's stream does not match" warning) - the add runs
    on the backward's own stream instead."""
    if g is None or p is None or g is _ACCUMULATED:
        return g
    acc = _grad_acc(p)
    if acc is None:
        return g
    acc.add_(g.reshape(acc.shape))
    return None


def _lin_param_grads(w, b, dz, x2, native, db=None):
    """(dW, db) of one Linear from its output-side gradient dz [T, N] and input x2.

    native: split-K MFMA GEMM accumulating dW (and db unless the caller already
    has it) into the fp32 .grad buffers in place (returns None grads).
    Otherwise fp32-output GEMM; db is taken from ``db`` when the caller already
    reduced it, else summed here."""
    if db is _ACCUMULATED:
        dw = _accumulate_wgrad(w, dz, x2, None)[0] if native else _mm_fp32(dz.t(), x2)
        return _into_grad(w, dw), None
    if native:
        if db is not None:
            dw, _ = _accumulate_wgrad(w, dz, x2, None)
            return _into_grad(w, dw), _into_grad(b, db)
        dw, db = _accumulate_wgrad(w, dz, x2, b)
        return _into_grad(w, dw), _into_grad(b, db)
    dw = _mm_fp32(dz.t(), x2)
    if b is not None and db is None:
        db = dz.float().sum(0)
    return _into_grad(w, dw), _into_grad(b, db)


def _dgrad(dz, w16, native):
    return get_ext().gemm_nn(dz, w16, wt=shadow_t(w16)) if native else dz @ w16


class _LinearFn(torch.autograd.Function):
    """y = act(x W^T + b) in bf16 with fp32 master weights.

    Native path: one MFMA GEMM with the bias/activation epilogue forward; in
    backward the activation derivative, one dgrad GEMM and one split-K wgrad
    GEMM that atomically accumulates dW and db into the fp32 ``.grad`` views of
    the flat gradient buffer (gradient-accumulation fusion).
    """

    @staticmethod
    def forward(ctx, x, w, b, w16, b16, act):
        shp = x.shape
        x2, T = _pad_rows(x.reshape(-1, shp[-1]), (w16.shape[0],))
        route = _route(x2, w16.shape[0], act)
        y, z, zact = _lin_fwd(x2, w16, b16, act, route)
        ctx.save_for_backward(x2, w16, z, y if act == "tanh" else None)
        ctx.params = (w, b)
        ctx.act = zact
        ctx.route = route
        ctx.shp = shp
        ctx.T = T
        return y[:T].reshape(*shp[:-1], w16.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w16, z, y = ctx.saved_tensors
        w, b = ctx.params
        dy2 = _pad_grad(dy.reshape(-1, dy.shape[-1]).contiguous(), x2.shape[0])
        _, nat_dgrad, nat_wgrad = ctx.route
        db = _take_db(dy2) if (b is not None and ctx.act == "none") else None
        if ctx.act != "none" or (b is not None and db is None and not nat_wgrad):
            # the activation backward reads dz anyway: it also sums db
            dz, db = _bias_act_bwd(dy2, z, y, ctx.act, b is not None)
        else:
            dz = dy2
        dx = _dgrad(dz, w16, nat_dgrad)[:ctx.T].reshape(ctx.shp) if ctx.needs_input_grad[0] else None
        dw, db = _lin_param_grads(w, b, dz, x2, nat_wgrad, db)
        return dx, dw, db, None, None, None


def linear(x, weight, bias=None, act="none"):
    """y = act(x @ W^T + b).  fp32 weights, compute in x.dtype."""
    if x.dtype == torch.float32:
        return _act_fwd(F.linear(x, weight, bias), act)
    return _LinearFn.apply(x, weight, bias, shadow(weight, x.dtype), shadow(bias, x.dtype), act)


def _dgrad_acc(dz, w16, native, dx_acc):
    """dx = dz @ W (+ dx_acc).  With hipBLASLt the residual-branch gradient is
    accumulated by the GEMM itself (beta = 1, in place on ``dx_acc``), which
    replaces autograd's separate bf16 add of the two branches."""
    if dx_acc is None:
        return _dgrad(dz, w16, native)
    if not native and dz.is_cuda:
        return dx_acc.addmm_(dz, w16)
    if native and get_ext().gemm_nn_acc_(dz, w16, dx_acc, wt=shadow_t(w16)):
        return dx_acc
    return dx_acc.add_(_dgrad(dz, w16, native))


def _res_gemm(x2, w16, b16, res, route, drop):
    """h = res + dropout(x2 W^T + b) in the GEMM epilogue (drop = (p, seed, offset)), or None
    when that path is off or the shape does not tile."""
    if not (_RES_FUSE and route[0] and drop is not None and res is not None):
        return None
    p, seed, off = drop
    return get_ext().gemm_nt_res(x2, w16, b16, res, float(p), seed, off)


def _mlp_fwd(x2, w1_16, b1_16, w2_16, b2_16, act, res=None, drop=None):
    """-> (y, h, z1, cfg, fused): fused = y is already res + dropout(fc2 output) (_res_gemm)."""
    r1 = _route(x2, w1_16.shape[0], act)
    h, z1, zact = _lin_fwd(x2, w1_16, b1_16, act, r1, q8=True)
    r2 = _route(h, w2_16.shape[0], "none")
    y = _res_gemm(h, w2_16, b2_16, res, r2, drop)
    fused = y is not None
    if not fused:
        y, _, _ = _lin_fwd(h, w2_16, b2_16, "none", r2)
    return y, h, z1, (zact, r1, r2), fused


def _mlp_bwd(dy2, x2, w1_16, w2_16, h, z1, params, cfg, need_dx, db2=None, dx_acc=None):
    """Backward of fc2(act(fc1(x))) -> (dx, dw1, db1, dw2, db2)."""
    w1, b1, w2, b2 = params
    act, r1, r2 = cfg
    # fc2 parameter grads
    if db2 is None and b2 is not None:
        db2 = _take_db(dy2)
    if b2 is not None and db2 is None and not r2[2]:
        _, db2 = _bias_act_bwd(dy2, None, None, "none", True)
    dw2, db2 = _lin_param_grads(w2, b2, dy2, h, r2[2], db2)
    # fc1 output gradient: activation backward (and fc1's bias gradient) fused into the
    # dgrad epilogue on the native route
    aux = h if act == "tanh" else z1
    dz1 = db1 = None
    if act != "none" and r2[1] and _gemm_shape_ok(dy2, w2_16.shape[1]):
        gb1 = _grad_acc(b1)
        slot = WGRAD_DEFER.bias_part(b1, gb1, dy2.shape[0], w2_16.shape[1]) if b1 is not None else None
        dz1, db1 = get_ext().gemm_nn_dact(dy2, w2_16, aux, _ACTS.index(act), b1 is not None, db_acc=gb1,
                                          part_out=slot, wt=shadow_t(w2_16))
        if dz1 is None:
            db1 = None
        elif gb1 is not None:
            db1 = _ACCUMULATED  # fc1's bias gradient went onto b1.grad (or its deferred slot)
    if dz1 is None:
        db1 = None
        if act == "deriv8":  # no fused dact GEMM for this shape: decode the codes
            z1, act = act_q8_decode(z1, dy2.shape[0], w2_16.shape[1]).to(dy2.dtype), "deriv"
        dh = _dgrad(dy2, w2_16, r2[1])
        if act != "none" or b1 is not None:
            # the activation backward reads dh anyway: it also sums db1
            dz1, db1 = _bias_act_bwd(dh, z1, h if act == "tanh" else None, act, b1 is not None)
        else:
            dz1 = dh
    dx = _dgrad_acc(dz1, w1_16, r1[1], dx_acc) if need_dx else None
    dw1, db1 = _lin_param_grads(w1, b1, dz1, x2, r1[2], db1)
    return dx, dw1, db1, dw2, db2


class _MLPFn(torch.autograd.Function):
    """y = fc2(act(fc1(x))) as one op, so the backward can fuse fc1's activation
    derivative into fc2's data-gradient GEMM epilogue (dz1 = (dy W2) * act'(z1)):
    the [T, ffn] hidden gradient is written once, already multiplied, instead of
    a dgrad GEMM followed by a separate activation-backward pass."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w1_16, b1_16, w2_16, b2_16, act):
        shp = x.shape
        x2, T = _pad_rows(x.reshape(-1, shp[-1]), (w1_16.shape[0], w2_16.shape[0]))
        y, h, z1, cfg, _ = _mlp_fwd(x2, w1_16, b1_16, w2_16, b2_16, act)
        ctx.save_for_backward(x2, w1_16, w2_16, h, z1)
        ctx.params = (w1, b1, w2, b2)
        ctx.cfg = cfg
        ctx.shp = shp
        ctx.T = T
        return y[:T].reshape(*shp[:-1], w2_16.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1_16, w2_16, h, z1 = ctx.saved_tensors
        dy2 = _pad_grad(dy.reshape(-1, dy.shape[-1]).contiguous(), x2.shape[0])
        dx, dw1, db1, dw2, db2 = _mlp_bwd(dy2, x2, w1_16, w2_16, h, z1, ctx.params, ctx.cfg,
                                          ctx.needs_input_grad[0])
        if dx is not None:
            dx = dx[:ctx.T].reshape(ctx.shp)
        return dx, dw1, db1, dw2, db2, None, None, None, None, None


def _ln_after_branch(y, x2, lw16, lb16, p, eps, seed, off, fused):
    """LayerNorm of a post-LN sublayer -> (out, hsave, mean, rstd, xo).

    fused: y already is h = x + dropout(branch) (the GEMM epilogue, pair-hash bits): the kernel
    reads h alone, and h itself is what the backward keeps.  Otherwise the kernel adds the
    dropped-out branch and the residual and writes the h copy."""
    ext = get_ext()
    if fused:
        out, _, mean, rstd = ext.add_ln_fwd(y, None, lw16, lb16, 0.0, float(eps), 0, 0, save_h=False)
        return out, y, mean, rstd, False
    out, hsave, mean, rstd = ext.add_ln_fwd(y, x2, lw16, lb16, float(p), float(eps), seed, off)
    return out, hsave, mean, rstd, False


class _MLPLNFn(torch.autograd.Function):
    """Post-LN FFN sublayer as one op: out = LN(dropout(fc2(act(fc1(x)))) + x).

    Owning both uses of x lets the backward hand the LayerNorm's residual
    gradient to fc1's dgrad GEMM as its accumulator (one GEMM writes
    dx = dres + dz1 W1) and the LN backward's column sum of dy to fc2 as its
    bias gradient - no autograd-side add of the two branch gradients."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, lw, lb, w1_16, b1_16, w2_16, b2_16, lw16, lb16, act, p, eps,
                seed, off):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y, h, z1, cfg, fused = _mlp_fwd(x2, w1_16, b1_16, w2_16, b2_16, act, res=x2, drop=(p, seed, off))
        out, hsave, mean, rstd, xo = _ln_after_branch(y, x2, lw16, lb16, p, eps, seed, off, fused)
        del y
        ctx.save_for_backward(x2, w1_16, w2_16, h, z1, out if xo else hsave, mean, rstd, lw16,
                              lb16 if xo else None, hsave if xo else None)
        ctx.params = (w1, b1, w2, b2)
        ctx.ln_params = (lw, lb)
        ctx.cfg = cfg
        ctx.ln = (p, seed, off, fused)
        ctx.shp = shp
        return out.reshape(shp)

    @staticmethod
    def backward(ctx, dout):
        x2, w1_16, w2_16, h, z1, hsave, mean, rstd, lw16, lb16, hcopy = ctx.saved_tensors
        p, seed, off, fused = ctx.ln
        need_dx = ctx.needs_input_grad[0]
        lw, lb = ctx.ln_params
        b2 = ctx.params[3]
        gb2 = _grad_acc(b2)
        dg, dbl = _grad_acc(lw), _grad_acc(lb)
        d2 = dout.reshape(-1, dout.shape[-1]).contiguous()
        part, pacc = (WGRAD_DEFER.ln_part(lw, d2.shape[0], d2.shape[1], dg, dbl, gb2)
                      if gb2 is not None else (None, False))
        dres, dy, dlw, dlb, dyb = get_ext().add_ln_bwd(
            d2, hsave, mean, rstd, lw16, float(p), seed, off, need_dx, True, True, dg_acc=dg, db_acc=dbl,
            dyb_acc=gb2, part_buf=part, part_acc=pacc, beta=lb16, hcopy=hcopy, pair_hash=fused)
        if b2 is not None and dyb is None:
            dyb = _ACCUMULATED  # fc2's bias gradient went onto b2.grad in the LN kernel
        dx, dw1, db1, dw2, db2 = _mlp_bwd(dy, x2, w1_16, w2_16, h, z1, ctx.params, ctx.cfg, need_dx,
                                          db2=dyb, dx_acc=dres)
        if dx is not None:
            dx = dx.reshape(ctx.shp)
        return (dx, dw1, db1, dw2, db2, _into_grad(lw, dlw), _into_grad(lb, dlb)) + (None,) * 11


class _AttnLNFn(torch.autograd.Function):
    """Post-LN self-attention sublayer as one op:
    out = LN(dropout(Wo attn(Wqkv x + bqkv) + bo) + x)   (bidirectional).

    Backward: LN backward (with the column sum of its dy = bo's gradient) ->
    out-proj dgrad/wgrad -> attention backward (with the column sum of dqkv =
    bqkv's gradient) -> qkv wgrad and a dgrad GEMM that accumulates onto the
    LN's residual gradient in place."""

    @staticmethod
    def forward(ctx, x, wq, bq, wo, bo, lw, lb, wq16, bq16, wo16, bo16, lw16, lb16, heads, p_attn,
                p, eps, seed_a, off_a, seed_l, off_l):
        shp = x.shape
        B, L, D = shp
        x2 = x.reshape(-1, D)
        rq = _route(x2, wq16.shape[0], "none")
        ext = get_ext()
        # head-major QKV (the L = 128 persistent attention): the GEMM epilogue stores
        # [B, 3H, L, 64], so both attention kernels read each head's Q / K / V block as
        # 16 KiB of contiguous memory instead of 128 rows strided by the token row
        hm = (_QKV_HEAD_MAJOR and rq[0] and x2.shape[0] % 256 == 0 and wq16.shape[0] % 256 == 0
              and ext.attn128_supports(L, D // heads, False))
        if hm:
            qkv, _, _ = ext.gemm_nt(x2, wq16, bq16, 0, False, L)
        else:
            qkv, _, _ = _lin_fwd(x2, wq16, bq16, "none", rq)
        qkv3 = qkv.view(B, L, wq16.shape[0])
        o, lse = ext.attn_fwd(qkv3, heads, float(p_attn), False, seed_a, off_a, bool(hm))
        o2 = o.view(-1, o.shape[-1])
        ro = _route(o2, wo16.shape[0], "none")
        y = _res_gemm(o2, wo16, bo16, x2, ro, (p, seed_l, off_l))
        fused = y is not None
        if not fused:
            y, _, _ = _lin_fwd(o2, wo16, bo16, "none", ro)
        out, hsave, mean, rstd, xo = _ln_after_branch(y, x2, lw16, lb16, p, eps, seed_l, off_l, fused)
        del y
        ctx.save_for_backward(x2, qkv3, o, lse, wq16, wo16, out if xo else hsave, mean, rstd,
                              lw16, lb16 if xo else None, hsave if xo else None)
        ctx.params = (wq, bq, wo, bo)
        ctx.ln_params = (lw, lb)
        ctx.cfg = (heads, p_attn, seed_a, off_a, p, seed_l, off_l, rq, ro, bool(hm), fused)
        ctx.shp = shp
        return out.reshape(shp)

    @staticmethod
    def backward(ctx, dout):
        x2, qkv3, o, lse, wq16, wo16, hsave, mean, rstd, lw16, lb16, hcopy = ctx.saved_tensors
        wq, bq, wo, bo = ctx.params
        heads, p_attn, seed_a, off_a, p, seed_l, off_l, rq, ro, hm, fused = ctx.cfg
        need_dx = ctx.needs_input_grad[0]
        ext = get_ext()
        lw, lb = ctx.ln_params
        dg, dbl, gbo = _grad_acc(lw), _grad_acc(lb), _grad_acc(bo)
        d2 = dout.reshape(-1, dout.shape[-1]).contiguous()
        part, pacc = (WGRAD_DEFER.ln_part(lw, d2.shape[0], d2.shape[1], dg, dbl, gbo)
                      if gbo is not None else (None, False))
        dres, dy, dlw, dlb, dyb = ext.add_ln_bwd(
            d2, hsave, mean, rstd, lw16, float(p), seed_l, off_l, need_dx, True, True, dg_acc=dg, db_acc=dbl,
            dyb_acc=gbo, part_buf=part, part_acc=pacc, beta=lb16, hcopy=hcopy, pair_hash=fused)
        if bo is not None and dyb is None:
            dyb = _ACCUMULATED  # the out projection's bias gradient went onto bo.grad
        # out projection
        o2 = o.view(-1, o.shape[-1])
        do = _dgrad(dy, wo16, ro[1])
        dwo, dbo = _lin_param_grads(wo, bo, dy, o2, ro[2], dyb if bo is not None else None)
        # attention
        gbq = _grad_acc(bq)
        apart = None
        if gbq is not None and WGRAD_DEFER.active and hasattr(ext, "attn_colpart_rows"):
            B_, L_ = qkv3.shape[0], qkv3.shape[1]
            D_ = qkv3.shape[-1] // (3 * heads)
            apart = WGRAD_DEFER.attn_part(bq, gbq, ext.attn_colpart_rows(B_, L_, heads, D_, False), heads, D_)
        kw = {"part_out": apart} if apart is not None else {}
        dqkv, dbq = ext.attn_bwd(do.view(o.shape), qkv3, o, lse, heads, float(p_attn), False, seed_a,
                                 off_a, bq is not None, hm, db_acc=gbq, **kw)  # dqkv comes back token-major
        if gbq is not None:
            dbq = _ACCUMULATED  # the column sums went straight onto bq.grad
        dz = dqkv.view(-1, dqkv.shape[-1])
        if bq is not None and dbq is None and not rq[2]:
            _, dbq = _bias_act_bwd(dz, None, None, "none", True)
        dx = _dgrad_acc(dz, wq16, rq[1], dres) if need_dx else None
        dwq, dbq = _lin_param_grads(wq, bq, dz, x2, rq[2], dbq)
        if dx is not None:
            dx = dx.reshape(ctx.shp)
        return (dx, dwq, dbq, dwo, dbo, _into_grad(lw, dlw), _into_grad(lb, dlb)) + (None,) * 14


def _ln_block_ok(x, *lins):
    if x.dtype != torch.bfloat16 or x.dim() != 3 or not native_ok(x, kernel="add_ln_fwd"):
        return False
    D = x.shape[-1]
    return D % 64 == 0 and D <= 2048 and all(lin.weight.dtype == torch.float32 for lin in lins)


def mlp_add_ln(x, fc1, fc2, ln, p=0.0, training=True):
    """Post-LN FFN sublayer LN(dropout(fc2(act(fc1(x)))) + x) as one fused op."""
    p = p if training else 0.0
    if not _ln_block_ok(x, fc1, fc2):
        f = mlp(x, fc1, fc2)
        return add_dropout_layernorm(f, x, ln.weight, ln.bias, p, ln.eps, training)
    dt = x.dtype
    seed, off = RNG.next()
    DB_HANDOFF_STATS["fused_sublayers"] += 1
    return _MLPLNFn.apply(x.contiguous(), fc1.weight, fc1.bias, fc2.weight, fc2.bias, ln.weight,
                          ln.bias, shadow(fc1.weight, dt), shadow(fc1.bias, dt), shadow(fc2.weight, dt),
                          shadow(fc2.bias, dt), shadow(ln.weight, dt), shadow(ln.bias, dt), fc1.act, p,
                          ln.eps, seed, off)


def attn_add_ln(x, qkv, out_proj, ln, heads, p_attn=0.0, p=0.0, training=True):
    """Post-LN bidirectional self-attention sublayer LN(dropout(Wo attn(Wqkv x)) + x) as one op."""
    p_attn = p_attn if training else 0.0
    p = p if training else 0.0
    B, L, D = x.shape if x.dim() == 3 else (0, 0, 0)
    if (not _ln_block_ok(x, qkv, out_proj) or qkv.act != "none" or out_proj.act != "none"
            or D % heads or D // heads not in (64, 128) or L % 64 or L > 1024
            or not native_ok(x, kernel="attn_fwd")):
        a = out_proj(attention(qkv(x), heads, p_attn, False, training))
        return add_dropout_layernorm(a, x, ln.weight, ln.bias, p, ln.eps, training)
    dt = x.dtype
    seed_a, off_a = RNG.next()
    seed_l, off_l = RNG.next()
    DB_HANDOFF_STATS["fused_sublayers"] += 1
    return _AttnLNFn.apply(x.contiguous(), qkv.weight, qkv.bias, out_proj.weight, out_proj.bias,
                           ln.weight, ln.bias, shadow(qkv.weight, dt), shadow(qkv.bias, dt),
                           shadow(out_proj.weight, dt), shadow(out_proj.bias, dt), shadow(ln.weight, dt),
                           shadow(ln.bias, dt), heads, p_attn, p, ln.eps, seed_a, off_a, seed_l, off_l)


def mlp(x, fc1, fc2):
    """fc2(act(fc1(x))) for two ``layers.Linear`` modules (fc1 carries the activation)."""
    if x.dtype == torch.float32 or not native_ok(x, kernel="gemm_nn_dact"):
        return fc2(fc1(x))
    dt = x.dtype
    return _MLPFn.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, shadow(fc1.weight, dt),
                        shadow(fc1.bias, dt), shadow(fc2.weight, dt), shadow(fc2.bias, dt), fc1.act)


# --------------------------------------------------------------------------- #
# LayerNorm, optionally fused with dropout(y) + residual add (post-LN BERT)
# --------------------------------------------------------------------------- #

class _AddLNFn(torch.autograd.Function):
    """out = LN(dropout(y) + residual) in one HIP kernel (fwd and bwd)."""

    @staticmethod
    def forward(ctx, y, residual, w, b, w16, b16, p, eps, seed, offset):
        out, hsave, mean, rstd = get_ext().add_ln_fwd(y, residual, w16, b16, float(p), float(eps),
                                                      seed, offset)
        ctx.save_for_backward(hsave, mean, rstd, w16)
        ctx.cfg = (p, seed, offset, residual is not None)
        ctx.wb = (w, b)
        return out

    @staticmethod
    def backward(ctx, dout):
        hsave, mean, rstd, w16 = ctx.saved_tensors
        p, seed, offset, has_res = ctx.cfg
        w, b = ctx.wb
        dres, dy, dw, db, dyb = get_ext().add_ln_bwd(dout.contiguous(), hsave, mean, rstd, w16,
                                                     float(p), seed, offset, has_res,
                                                     ctx.needs_input_grad[0], ctx.needs_input_grad[0],
                                                     dg_acc=_grad_acc(w), db_acc=_grad_acc(b))
        if dy is not None:
            _offer_db(dy, dyb)
        return dy, (dres if has_res else None), _into_grad(w, dw), _into_grad(b, db), None, None, None, None, None, None


class _AddLNExFn(torch.autograd.Function):
    """(out, h) with h = dropout(y [+ pos] [+ temb]) + residual and out = LN(h) (post:
    h = y + pos + temb + residual, out = dropout(LN(h))) in one kernel; h is an
    output of its own (the pre-LN residual stream), whose incoming gradient the
    backward kernel adds to the LN gradient.  pos: [L, H] broadcast over the batch,
    temb: [B, H] broadcast over the sequence (their gradients are the batch / sequence
    sums of dy, reduced in fp32)."""

    @staticmethod
    def forward(ctx, y, residual, pos, temb, w, b, w16, b16, p, eps, seed, offset, post, L):
        # pos / temb arrive in their own dtype (an fp32 position-embedding parameter slice
        # keeps an fp32 gradient: its batch sum is never rounded to bf16); the kernel
        # reads compute-dtype copies
        ctx.pt_dtypes = (None if pos is None else pos.dtype, None if temb is None else temb.dtype)
        pos = None if pos is None else pos.to(y.dtype).contiguous()
        temb = None if temb is None else temb.to(y.dtype).contiguous()
        out, hsave, mean, rstd = get_ext().add_ln_fwd(y, residual, w16, b16, float(p), float(eps), seed,
                                                      offset, pos, temb, int(L), bool(post))
        ctx.save_for_backward(hsave, mean, rstd, w16)
        ctx.cfg = (p, seed, offset, residual is not None, pos is not None, temb is not None, post, L)
        ctx.wb = (w, b)
        ctx.set_materialize_grads(False)  # an unused h (last layer, input block) costs nothing
        return out, hsave

    @staticmethod
    def backward(ctx, dout, dh):
        hsave, mean, rstd, w16 = ctx.saved_tensors
        p, seed, offset, has_res, has_pos, has_temb, post, L = ctx.cfg
        ng = ctx.needs_input_grad
        need_dy = ng[0] or (has_pos and ng[2]) or (has_temb and ng[3])
        if dout is None:
            dout = torch.zeros_like(hsave)
        w, b = ctx.wb
        dg, dbl = _grad_acc(w), _grad_acc(b)
        dout = dout.contiguous()
        part, pacc = WGRAD_DEFER.ln_part(w, dout.shape[0], dout.shape[1], dg, dbl, None)
        dres, dy, dw, db, _ = get_ext().add_ln_bwd(
            dout, hsave, mean, rstd, w16, float(p), seed, offset, has_res and ng[1], need_dy,
            False, dh_in=None if dh is None else dh.contiguous(), post=bool(post),
            dg_acc=dg, db_acc=dbl, part_buf=part, part_acc=pacc)
        dpos = dtemb = None
        if need_dy:
            H = dy.shape[-1]
            want_p, want_t = bool(has_pos and ng[2]), bool(has_temb and ng[3])
            # both sums from one read of dy (csrc/norm.hip seq_pos_partial_kernel)
            sums = (get_ext().seq_pos_sums(dy, int(L), want_p, want_t)
                    if (want_p or want_t) and hasattr(get_ext(), "seq_pos_sums") else [])
            if sums:
                if want_p:
                    dpos = sums[0].to(ctx.pt_dtypes[0])
                if want_t:
                    dtemb = sums[1].to(ctx.pt_dtypes[1])
            else:
                d3 = dy.view(-1, L, H)
                if want_p:
                    dpos = torch.sum(d3, 0, dtype=torch.float32).to(ctx.pt_dtypes[0])
                if want_t:
                    dtemb = torch.sum(d3, 1, dtype=torch.float32).to(ctx.pt_dtypes[1])
        return ((dy if ng[0] else None), (dres if has_res else None), dpos, dtemb, dw, db,
                None, None, None, None, None, None, None, None)


def _add_ln_ex(y, residual, pos, temb, weight, bias, p, eps, training, post):
    """Shared front of :func:`embed_layernorm` / :func:`residual_layernorm` -> (out, h)."""
    p = p if training else 0.0
    B, L, H = y.shape
    if (y.dtype == torch.bfloat16 and native_ok(y, kernel="add_ln_fwd") and H % 64 == 0 and H <= 2048):
        seed, off = RNG.next()
        out, h = _AddLNExFn.apply(
            y.reshape(-1, H).contiguous(),
            None if residual is None else residual.reshape(-1, H).contiguous(),
            None if pos is None else pos.reshape(L, H),
            None if temb is None else temb.reshape(B, H),
            weight, bias, shadow(weight, y.dtype), shadow(bias, y.dtype), p, eps, seed, off, post, L)
        return out.view(B, L, H), h.view(B, L, H)
    s_ = y
    if pos is not None:
        s_ = s_ + pos.reshape(1, L, H).to(y.dtype)
    if temb is not None:
        s_ = s_ + temb.reshape(B, 1, H).to(y.dtype)
    h = F.dropout(s_, p, True) if (p > 0 and not post) else s_
    if residual is not None:
        h = h + residual
    out = (F.layer_norm(h, (H,), weight, bias, eps) if h.dtype == torch.float32
           else _LNTorchFn.apply(h, weight, bias, eps))
    if p > 0 and post:
        out = F.dropout(out, p, True)
    return out, h


def embed_layernorm(y, pos, temb, weight, bias, p=0.0, eps=1e-12, training=True):
    """dropout(LN(y + pos + temb)): the DiffuSeq input block (reference model:
    ``Dropout(LayerNorm(up_proj(x) + pos_emb + time_emb))``) in one kernel.
    y: [B, L, H]; pos: [1, L, H] / [L, H]; temb: [B, H]."""
    return _add_ln_ex(y, None, pos, temb, weight, bias, p, eps, training, post=True)[0]


def residual_layernorm(h, x, weight, bias, p=0.0, eps=1e-5, training=True, pos=None):
    """Pre-LN residual step -> (x_new, LN(x_new)) with x_new = x + dropout(h [+ pos])
    (x may be None: the GPT-2 input, h = token + position embeddings)."""
    ln, xn = _add_ln_ex(h, x, pos, None, weight, bias, p, eps, training, post=False)
    return xn, ln


class RNG:
    """(seed, offset) of the in-kernel Philox streams.

    Eager runs: the offset is a host counter that advances per call site, so every launch
    draws fresh numbers.  HIP-graph replays (utils/trainer.py graph mode): the offsets are
    baked into the captured launches, and every kernel adds a device-side base
    (csrc/common.h ``g_rng_base``, 0 in eager runs).  ``graph_begin`` sets the base so a
    replay of a graph captured at offsets [r0, r0 + span) draws [counter, counter + span) -
    exactly what an eager step would have drawn next - and ``graph_end`` resets it to 0."""
    seed = 1234
    counter = 0
    _dev_base = 0

    @classmethod
    def next(cls, n=1):
        off = cls.counter
        cls.counter += n
        return cls.seed, off

    @classmethod
    def graph_begin(cls, r0, span):
        d = (cls.counter - r0) & 0xFFFFFFFF
        get_ext().rng_base_add(d)
        cls._dev_base = d
        cls.counter += span

    @classmethod
    def graph_end(cls):
        if cls._dev_base:
            get_ext().rng_base_add((-cls._dev_base) & 0xFFFFFFFF)
            cls._dev_base = 0


def add_dropout_layernorm(y, residual, weight, bias, p=0.0, eps=1e-12, training=True):
    """LN(dropout(y) + residual) (residual may be None)."""
    p = p if training else 0.0
    if y.dtype == torch.bfloat16 and native_ok(y, kernel="add_ln_fwd") and y.shape[-1] % 64 == 0 and y.shape[-1] <= 2048:
        seed, off = RNG.next()
        shp = y.shape
        out = _AddLNFn.apply(y.reshape(-1, shp[-1]).contiguous(),
                             None if residual is None else residual.reshape(-1, shp[-1]).contiguous(),
                             weight, bias, shadow(weight, y.dtype), shadow(bias, y.dtype),
                             p, eps, seed, off)
        return out.reshape(shp)
    h = F.dropout(y, p, True) if p > 0 else y
    if residual is not None:
        h = h + residual
    if h.dtype == torch.float32:
        return F.layer_norm(h, (h.shape[-1],), weight, bias, eps)
    return _LNTorchFn.apply(h, weight, bias, eps)


class _LNTorchFn(torch.autograd.Function):
    """Reference LN for bf16 activations with fp32 weight grads (non-native path)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        xf = x.float()
        mu = xf.mean(-1, keepdim=True)
        var = ((xf - mu) ** 2).mean(-1, keepdim=True)
        rstd = torch.rsqrt(var + eps)
        xhat = (xf - mu) * rstd
        out = xhat * w + b
        ctx.save_for_backward(xhat, rstd, w)
        return out.to(x.dtype)

    @staticmethod
    def backward(ctx, dout):
        xhat, rstd, w = ctx.saved_tensors
        g = dout.float()
        d = g.shape[-1]
        dw = (g * xhat).reshape(-1, d).sum(0)
        db = g.reshape(-1, d).sum(0)
        gx = g * w
        dx = rstd * (gx - gx.mean(-1, keepdim=True) - xhat * (gx * xhat).mean(-1, keepdim=True))
        return dx.to(dout.dtype), dw, db, None


def layer_norm(x, weight, bias, eps=1e-12):
    return add_dropout_layernorm(x, None, weight, bias, 0.0, eps, training=False)


# --------------------------------------------------------------------------- #
# Attention (bidirectional or causal), qkv packed [B, L, 3, H, D]
# --------------------------------------------------------------------------- #

class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_heads, p, causal, seed, offset):
        out, lse = get_ext().attn_fwd(qkv, n_heads, float(p), bool(causal), seed, offset)
        ctx.save_for_backward(qkv, out, lse)
        ctx.cfg = (n_heads, p, causal, seed, offset)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        n_heads, p, causal, seed, offset = ctx.cfg
        dqkv, db = get_ext().attn_bwd(dout.contiguous(), qkv, out, lse, n_heads, float(p),
                                      bool(causal), seed, offset, True)
        _offer_db(dqkv, db)
        return dqkv, None, None, None, None, None


def attention(qkv, n_heads, p=0.0, causal=False, training=True):
    """qkv: [B, L, 3*H*D] packed projection output -> [B, L, H*D]."""
    p = p if training else 0.0
    B, L, three_hd = qkv.shape
    hd = three_hd // 3
    D = hd // n_heads
    if (qkv.dtype == torch.bfloat16 and native_ok(qkv, kernel="attn_fwd") and D in (64, 128)
            and L % 64 == 0 and L <= 1024):
        seed, off = RNG.next()
        return _AttnFn.apply(qkv.contiguous(), n_heads, p, causal, seed, off)
    q, k, v = qkv.view(B, L, 3, n_heads, D).permute(2, 0, 3, 1, 4).unbind(0)
    o = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=causal)
    return o.transpose(1, 2).reshape(B, L, hd)


# --------------------------------------------------------------------------- #
# Fused linear + cross-entropy (tied lm_head), per-token loss
# --------------------------------------------------------------------------- #

# the fused CE weight gradient accumulates straight into the tied weight's flat fp32 .grad
_XENT_GRAD_ACC = True


class _LinearXentFn(torch.autograd.Function):
    """Per-token CE of x @ W^T + b, logits never materialised (csrc/xent.hip).  When x
    needs a gradient the forward also produces the unscaled input gradient
    dxu = softmax . W - W[target] in the same vocabulary sweep (fp32, [N, E]), so the
    backward's dx is one multiply by the upstream per-token gradient instead of a
    second pass over all N x V logits."""

    @staticmethod
    def forward(ctx, x, w, b, w16, b16, target):
        ext = get_ext()
        ctx.dxu = None
        if ctx.needs_input_grad[0] and _XENT_FUSED_DX and hasattr(ext, "lxent_fwd_dx"):
            loss, lse, ctx.dxu = ext.lxent_fwd_dx(x, w16, b16, target)
        else:
            loss, lse = ext.lxent_fwd(x, w16, b16, target)
        ctx.save_for_backward(x, w16, b16, target, lse)
        ctx.has_b = b is not None
        ctx.wb = (w, b)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        x, w16, b16, target, lse = ctx.saved_tensors
        dxu, ctx.dxu = ctx.dxu, None
        g = dloss.contiguous().float()
        need_dx = ctx.needs_input_grad[0] and dxu is None
        w, b = ctx.wb
        need_dw, need_db = ctx.needs_input_grad[1], ctx.has_b and ctx.needs_input_grad[2]
        # straight into the flat fp32 .grad buffers when they exist (the kernel's partials are
        # atomics: no zero-filled [V, E] scratch and no add per call)
        acc = _XENT_GRAD_ACC
        gw, gb = (_grad_acc(w) if need_dw and acc else None), (_grad_acc(b) if need_db and acc else None)
        dx, dw, db = get_ext().lxent_bwd(g, x, w16, b16, target, lse, need_dx, need_dw, need_db,
                                         _XENT_ONEHOT_SCATTER, dw_acc=gw, db_acc=gb)
        if dxu is not None:
            dx = dxu.mul_(g.unsqueeze(1)).to(x.dtype)
        return (dx, None if (need_dw and gw is not None) else _into_grad(w, dw),
                None if (need_db and gb is not None) else _into_grad(b, db), None, None, None)


def _pad_vocab(w16, b16, mult=256):
    """Vocabulary rows padded to a multiple of ``mult`` (zero rows; their logits are
    masked by the row kernels), so every logits row is 16-byte aligned and the
    weight-gradient GEMM tiles."""
    V = w16.shape[0]
    Vp = (V + mult - 1) // mult * mult
    if Vp == V:
        return w16, b16
    wp = torch.zeros(Vp, w16.shape[1], dtype=w16.dtype, device=w16.device)
    wp[:V].copy_(w16)
    bp = None
    if b16 is not None:
        bp = torch.zeros(Vp, dtype=b16.dtype, device=b16.device)
        bp[:V].copy_(b16)
    return wp, bp


def _chunk_logits(xc, wp, bp, out=None):
    """[chunk, Vp] logits of one token chunk on the persistent MFMA GEMM (bias fused,
    written straight into ``out`` - a row slice of the [N, Vp] buffer - when given)."""
    if out is None:
        out = torch.empty(xc.shape[0], wp.shape[0], dtype=xc.dtype, device=xc.device)
    get_ext().gemm_nt_into(xc, wp, bp, out)
    return out


class _ChunkedLinearXentFn(torch.autograd.Function):
    """Per-token CE for WIDE inputs (E > 256, e.g. GPT-2's 768 x 50257 LM head).

    All three GEMMs run on the hand-written gfx950 kernels (csrc/gemm256.hip): the logits
    of one token chunk at a time (bias fused) into a [chunk, Vp] bf16 buffer, which the
    row kernels of ``csrc/xent_rows.hip`` turn into (loss, lse) and - when the logits are
    kept for the backward - into softmax - onehot in place; backward dx = dlogits W
    (data-gradient GEMM, K = Vp) and dW = dlogits^T (g x) (split-K weight-gradient GEMM
    over all tokens at once).  The vocabulary is padded to a multiple of 256 once per
    forward (the padded weight is reused by the backward) and the token count to a
    multiple of 256 (padded tokens have target -1: zero loss, zero gradient rows)."""

    @staticmethod
    def forward(ctx, x, w, b, w16, b16, target, chunk):
        ext = get_ext()
        ctx.wb = (w, b)
        N0, V = x.shape[0], w16.shape[0]
        N = (N0 + 255) // 256 * 256
        if N != N0:  # token rows padded to the GEMM tile (zero rows, ignored targets)
            xp = torch.zeros(N, x.shape[1], dtype=x.dtype, device=x.device)
            xp[:N0].copy_(x)
            tp = torch.full((N,), -1, dtype=target.dtype, device=target.device)
            tp[:N0].copy_(target)
            x, target = xp, tp
        wp, bp = _pad_vocab(w16, b16)
        loss = torch.empty(N, dtype=torch.float32, device=x.device)
        lse = torch.empty(N, dtype=torch.float32, device=x.device)
        # 288 GB of HBM: keep the bf16 logits for the backward (which then needs no logits
        # GEMM of its own) when they fit the budget
        keep = any(ctx.needs_input_grad[:3]) and N * wp.shape[0] * 2 <= _XENT_KEEP_BYTES
        # kept logits: one row pass leaves softmax - onehot (unscaled) in place of the
        # logits (xent_rows_fwd_grad_), so the backward needs no row pass of its own; all
        # chunks are row slices of ONE [N, Vp] buffer, so the backward's weight gradient is
        # a single split-K GEMM over all N tokens
        kept_is_grad = keep and _XENT_ROWS_FUSED
        allg = torch.empty(N, wp.shape[0], dtype=x.dtype, device=x.device) if keep else None
        if kept_is_grad:
            # kept chunks (_XENT_FWD_CHUNK_BYTES): the backward's GEMMs run over all N tokens at
            # once, so the forward chunk size is free
            chunk = min(chunk, max(256, (_XENT_FWD_CHUNK_BYTES // (wp.shape[0] * 2)) // 256 * 256))
        for s in range(0, N, chunk):
            e = min(N, s + chunk)
            lg = _chunk_logits(x[s:e], wp, bp, allg[s:e] if allg is not None else None)
            # the row kernels write this chunk's slices of loss / lse directly
            if kept_is_grad:
                res = ext.xent_rows_fwd_grad_(lg, V, target[s:e], loss[s:e], lse[s:e])
                assert res, "xent_rows_fwd_grad_ refused the row length"
            else:
                ext.xent_rows_fwd(lg, V, target[s:e], loss[s:e], lse[s:e])
        ctx.allg = allg
        ctx.kept_is_grad = kept_is_grad
        ctx.save_for_backward(x, w16, b16, target, lse, wp, bp)
        ctx.params = (w, b)
        ctx.chunk = chunk
        ctx.n0 = N0
        return loss[:N0]

    @staticmethod
    def backward(ctx, dloss):
        x, w16, b16, target, lse, wp, bp = ctx.saved_tensors
        w, b = ctx.params
        ext = get_ext()
        N, E, V = x.shape[0], x.shape[1], w16.shape[0]
        N0 = ctx.n0
        Vp = wp.shape[0]
        g_all = torch.zeros(N, dtype=torch.float32, device=x.device)
        g_all[:N0].copy_(dloss)
        need_dx, need_dw, need_db = ctx.needs_input_grad[0], ctx.needs_input_grad[1], (
            b is not None and ctx.needs_input_grad[2])
        dx = torch.empty_like(x) if need_dx else None
        dwp = torch.zeros(Vp, E, dtype=torch.float32, device=x.device) if need_dw else None
        db = torch.zeros(V, dtype=torch.float32, device=x.device) if need_db else None
        allg, ctx.allg = ctx.allg, None
        unscaled = allg is not None and ctx.kept_is_grad
        all_n = unscaled and _XENT_DX_ALL
        if all_n:
            # kept softmax - onehot for all N tokens: dx = diag(g) (G Wp) as ONE data-gradient
            # GEMM (a per-chunk GEMM has only chunk/256 x 3 output tiles at E = 768)
            if need_dx:
                ext.gemm_nn_into(allg, wp, dx)
                dx.mul_(g_all[:, None])
            if need_db:
                for s in range(0, N, ctx.chunk):
                    e = min(N, s + ctx.chunk)
                    db.add_(g_all[s:e] @ allg[s:e, :V].float())
        for s in range(0, N if not all_n else 0, ctx.chunk):
            e = min(N, s + ctx.chunk)
            # a kept chunk is a row slice of allg: it is freed with the whole buffer at
            # the end of the backward, not per chunk
            dlg = allg[s:e] if allg is not None else _chunk_logits(x[s:e], wp, bp)
            g = g_all[s:e]
            if not unscaled:
                ext.xent_rows_bwd_(dlg, V, target[s:e], lse[s:e], g)
            if need_dx:
                ext.gemm_nn_into(dlg, wp, dx[s:e])
                if unscaled:  # dlg = softmax - onehot: the upstream gradient scales rows
                    dx[s:e].mul_(g[:, None])
            if need_dw and allg is None:
                ext.gemm_wgrad(dlg, x[s:e] if not unscaled else (x[s:e] * g[:, None]).to(x.dtype), dwp, None)
            if need_db:
                db.add_((g @ dlg[:, :V].float()) if unscaled else dlg[:, :V].float().sum(0))
        if need_dw and allg is not None:
            # dW = G^T (diag(g) x) over all N tokens as one split-K GEMM
            ext.gemm_wgrad(allg, (x * g_all[:, None]).to(x.dtype) if unscaled else x, dwp, None)
        del allg
        dw = dwp[:V] if need_dw else None
        if dx is not None and N != N0:
            dx = dx[:N0]
        w, b = ctx.wb
        return dx, _into_grad(w, dw), _into_grad(b, db), None, None, None, None


# wide-E CE: kept logit chunks become softmax - onehot in the forward's row pass
_XENT_ROWS_FUSED = True

# fused CE backward, _XENT_ONEHOT_SCATTER: the weight-gradient kernel computes softmax only
# and the target one-hot goes in as a sorted scatter. Off by default: the kernel saves 0.35
# ms/step but the scatter and the bias index_add cost 1.7 (profiles/xent_onehot_scatter_ab_r4.txt)
_XENT_ONEHOT_SCATTER = False

# fused CE: forward also emits the unscaled input gradient (False: separate dx pass)
_XENT_FUSED_DX = True

# tokens per logits chunk of the wide-E path: about 2 GiB of bf16 logits (fewer, larger
# GEMMs: GPT-2 bs128 171 -> 162 ms/step against 0.5 GiB chunks)
_XENT_CHUNK_BYTES = 2048 << 20
# logits kept from the forward for the backward (bytes; GPT-2 small at 128 x 1024 tokens
# needs 13 GB): above this the backward recomputes each chunk
_XENT_KEEP_BYTES = 24 << 30
# kept logits: the backward's dx as one GEMM over all tokens (False: per chunk)
_XENT_DX_ALL = True
# forward chunk when the logits are kept (softmax - onehot in place).  128 MB chunks (resident
# in the 256 MB Infinity Cache) did not speed the row pass up (profiles/gpt2_head_ab_r4.txt) and
# cost ~200 small loss/lse copies per GPT-2 step, so the default keeps the 2 GB chunks
_XENT_FWD_CHUNK_BYTES = 2048 << 20


def linear_cross_entropy(x, weight, bias, target):
    """Per-token CE of logits = x @ W^T + b against ``target`` without materialising logits.

    x: [N, E]; weight: [V, E]; target: [N] int64 -> loss [N] fp32.  E in {128, 256}:
    fully fused MFMA kernels (csrc/xent.hip); wider E: chunked logits on the persistent
    MFMA GEMM + row kernels (csrc/xent_rows.hip).
    """
    if x.dtype == torch.bfloat16 and native_ok(x, kernel="lxent_fwd") and x.shape[-1] in (128, 256):
        return _LinearXentFn.apply(x.contiguous(), weight, bias, shadow(weight, x.dtype),
                                   shadow(bias, x.dtype), target.contiguous())
    if x.dtype == torch.bfloat16 and native_ok(x, kernel="xent_rows_fwd") and x.dim() == 2:
        Vp = (weight.shape[0] + 255) // 256 * 256
        chunk = max(256, (_XENT_CHUNK_BYTES // (Vp * 2)) // 256 * 256)
        return _ChunkedLinearXentFn.apply(x.contiguous(), weight, bias, shadow(weight, x.dtype),
                                          shadow(bias, x.dtype), target.contiguous(), chunk)
    logits = linear(x, weight, bias)
    return F.cross_entropy(logits.float(), target, reduction="none")


# --------------------------------------------------------------------------- #
# Embedding gather with fp32 weight grad
# --------------------------------------------------------------------------- #

class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, w16):
        ctx.save_for_backward(ids)
        ctx.n = w.shape[0]
        ctx.w = w
        return F.embedding(ids, w16)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        if native_ok(dy, kernel="emb_grad") and dy.shape[-1] in (128, 256, 768, 1024, 2048):
            # sorted segment sum on the device (csrc/diffusion.hip), no ATen index_add; its
            # atomics add straight onto the flat fp32 .grad view when there is one
            acc = _grad_acc(ctx.w)
            dw = acc if acc is not None else torch.zeros(ctx.n, dy.shape[-1], dtype=torch.float32,
                                                         device=dy.device)
            get_ext().emb_grad(ids.contiguous(), dy.contiguous(), dw)
            return None, (None if acc is not None else dw), None
        dw = torch.zeros(ctx.n, dy.shape[-1], dtype=torch.float32, device=dy.device)
        dw.index_add_(0, ids.reshape(-1), dy.reshape(-1, dy.shape[-1]).float())
        return None, _into_grad(ctx.w, dw), None


def embedding(ids, weight, dtype):
    if dtype == torch.float32:
        return F.embedding(ids, weight)
    return _EmbFn.apply(ids, weight, shadow(weight, dtype))


def timestep_embedding(timesteps, dim, max_period=10000, dtype=None):
    """Sinusoidal embedding [cos | sin] (DiffuSeq / guided-diffusion convention).

    bf16 on a HIP device: one kernel writes the bf16 embedding (csrc/diffusion.hip)."""
    if dtype == torch.bfloat16 and native_ok(timesteps, kernel="timestep_emb"):
        return get_ext().timestep_emb(timesteps.float().contiguous(), int(dim), float(max_period))
    emb = _timestep_embedding_ref(timesteps, dim, max_period)
    return emb if dtype is None else emb.to(dtype)


def _timestep_embedding_ref(timesteps, dim, max_period=10000):
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) *
                      torch.arange(half, dtype=torch.float32, device=timesteps.device) / half)
    args = timesteps[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb
