"""Fused dropout+residual+LayerNorm and bias+activation HIP kernels vs PyTorch fp32."""
import pytest
import torch

from distributed_pipeline_amd.ops import nn as ops

pytestmark = pytest.mark.gpu


def _ext():
    from distributed_pipeline_amd.ops._ext import get_ext
    return get_ext(required=True)


@pytest.mark.parametrize("R,D,res", [(1000, 768, True), (37, 128, False), (4096, 2048, True), (64, 64, True),
                                     (70000, 2048, True), (3000, 1536, False), (70000, 768, True),
                                     (40000, 768, True)])  # 40000: the capped small-R grid
def test_add_ln_no_dropout(R, D, res):
    torch.manual_seed(0)
    y = torch.randn(R, D, device="cuda").bfloat16()
    r = torch.randn(R, D, device="cuda").bfloat16() if res else None
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(D, device="cuda")).bfloat16()
    out, hs, mean, rstd = _ext().add_ln_fwd(y, r, g, b, 0.0, 1e-12, 1, 0)
    h = y.float() + (r.float() if res else 0)
    h = h.bfloat16().float().requires_grad_(True)
    gf = g.float().requires_grad_(True)
    bf = b.float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(h, (D,), gf, bf, 1e-12)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    dout = torch.randn(R, D, device="cuda").bfloat16()
    ref.backward(dout.float())
    dres, dy, dg, db, dyb = _ext().add_ln_bwd(dout, hs, mean, rstd, g, 0.0, 1, 0, res, True, True)
    torch.testing.assert_close(dy.float(), h.grad, rtol=2e-2, atol=2e-2)
    ref_dyb = dy.float().sum(0)  # column sums of the emitted bf16 dy (next layer's bias grad)
    torch.testing.assert_close(dyb, ref_dyb, rtol=1e-3, atol=1e-3 * ref_dyb.abs().max().item())
    if res:
        torch.testing.assert_close(dres.float(), h.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dg, gf.grad, rtol=1e-2, atol=1e-2 * gf.grad.abs().max().item())
    torch.testing.assert_close(db, bf.grad, rtol=1e-2, atol=1e-2 * bf.grad.abs().max().item())


@pytest.mark.parametrize("R,D,p", [(1000, 768, 0.0), (70000, 768, 0.1), (4096, 2048, 0.1), (70000, 2048, 0.0),
                                   (3000, 1536, 0.1), (256, 1024, 0.1)])
def test_add_ln_bwd_from_output(R, D, p):
    """Output-based LayerNorm backward (forward with h_guard: no h copy written; backward given
    beta and the LN output: xhat = (out - beta) / gamma) vs the fp32 PyTorch LayerNorm of the
    same bf16 h with the pre-LN dropout mask regenerated, judged against the h-copy backward's
    own bf16 error.  Then the guard: one |gamma| < 0.125 makes the forward write the h copy
    and the backward take the h-copy path - the unguarded kernels' results."""
    ext = _ext()
    torch.manual_seed(0)
    y = torch.randn(R, D, device="cuda").bfloat16()
    r = torch.randn(R, D, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(D, device="cuda")).clamp(min=0.6).bfloat16()
    b = (0.2 * torch.randn(D, device="cuda")).clamp(-0.5, 0.5).bfloat16()  # |b| < |g|: unguarded
    out, hs, mean, rstd = ext.add_ln_fwd(y, r, g, b, p, 1e-12, 3, 9)
    hc = torch.full_like(hs, float("nan"))  # the guarded copy must stay unwritten and unread
    out2, hs2, mean2, rstd2 = ext.add_ln_fwd(y, r, g, b, p, 1e-12, 3, 9, h_guard=True)
    assert torch.equal(out, out2) and torch.equal(rstd, rstd2) and torch.equal(mean, mean2)
    dout = torch.randn(R, D, device="cuda").bfloat16()
    ref = ext.add_ln_bwd(dout, hs, mean, rstd, g, p, 3, 9, True, True, True)
    got = ext.add_ln_bwd(dout, out, mean, rstd, g, p, 3, 9, True, True, True, beta=b, hcopy=hc)
    h = hs.float().requires_grad_(True)
    gf = g.float().requires_grad_(True)
    bf = b.float().requires_grad_(True)
    torch.nn.functional.layer_norm(h, (D,), gf, bf, 1e-12).backward(dout.float())
    dy_ref = h.grad * (ref[1] != 0).float() / (1 - p)
    assert torch.equal(got[1] == 0, ref[1] == 0)  # dy: same dropout mask
    for k, want in ((0, h.grad), (1, dy_ref)):
        e_got = (got[k].float() - want).abs()
        e_ref = (ref[k].float() - want).abs()
        assert e_got.max().item() <= 2 * e_ref.max().item() + 1e-2, (k, e_got.max().item(), e_ref.max().item())
        assert e_got.mean().item() <= 1.5 * e_ref.mean().item() + 1e-4, (k, e_got.mean().item(), e_ref.mean().item())
    for k, want in ((2, gf.grad), (3, bf.grad), (4, ref[4])):
        torch.testing.assert_close(got[k], want, rtol=1e-2, atol=1e-2 * want.abs().max().item())
    # guard: a small gamma entry, or a column with |beta| > |gamma|, -> the h copy is written
    # and read, results == h-copy kernels
    gs = g.clone()
    gs[5] = 0.01
    out3, hs3, mean3, rstd3 = ext.add_ln_fwd(y, r, gs, b, p, 1e-12, 3, 9)
    _, hg, _, _ = ext.add_ln_fwd(y, r, gs, b, p, 1e-12, 3, 9, h_guard=True)
    assert torch.equal(hg, hs3)
    ref3 = ext.add_ln_bwd(dout, hs3, mean3, rstd3, gs, p, 3, 9, True, True, True)
    got3 = ext.add_ln_bwd(dout, out3, mean3, rstd3, gs, p, 3, 9, True, True, True, beta=b, hcopy=hg)
    for a, e in zip(got3, ref3):  # same math, other template instance (contraction may differ)
        if e is None:
            assert a is None
        elif e.dtype == torch.bfloat16:
            torch.testing.assert_close(a.float(), e.float(), rtol=8e-3, atol=1e-3 * e.float().abs().max().item())
        else:
            torch.testing.assert_close(a, e, rtol=1e-4, atol=1e-4 * e.abs().max().item())
    bs = b.clone()
    bs[7] = 1.5 * g[7].float()
    _, hgb, _, _ = ext.add_ln_fwd(y, r, g, bs, p, 1e-12, 3, 9, h_guard=True)
    _, hsb, _, _ = ext.add_ln_fwd(y, r, g, bs, p, 1e-12, 3, 9)
    assert torch.equal(hgb, hsb), "a |beta| > |gamma| column must keep the h copy"


@pytest.mark.parametrize("gmin", [0.13, 0.25, 0.5])
@pytest.mark.parametrize("bscale", [0.1, 0.5, 2.0])
def test_add_ln_bwd_from_output_guard_region(gmin, bscale):
    """The output-based backward (or its guard) over gamma spreads down to min |gamma| in
    {0.13, 0.25, 0.5} and realistic-to-large beta: every combination must be as accurate as
    the h-copy backward against the fp32 LayerNorm of the same bf16 h (the guard sends the
    columns / layers where (out - beta) / gamma would amplify out's rounding to the h copy)."""
    ext = _ext()
    torch.manual_seed(1)
    R, D, p = 4096, 768, 0.1
    y = torch.randn(R, D, device="cuda").bfloat16()
    r = torch.randn(R, D, device="cuda").bfloat16()
    g = (gmin + (1.5 - gmin) * torch.rand(D, device="cuda"))
    g = (g * torch.where(torch.rand(D, device="cuda") < 0.5, -1.0, 1.0)).bfloat16()
    b = (bscale * torch.randn(D, device="cuda")).bfloat16()
    out, hs, mean, rstd = ext.add_ln_fwd(y, r, g, b, p, 1e-12, 5, 2)
    _, hg, _, _ = ext.add_ln_fwd(y, r, g, b, p, 1e-12, 5, 2, h_guard=True)
    dout = torch.randn(R, D, device="cuda").bfloat16()
    ref = ext.add_ln_bwd(dout, hs, mean, rstd, g, p, 5, 2, True, True, True)
    got = ext.add_ln_bwd(dout, out, mean, rstd, g, p, 5, 2, True, True, True, beta=b, hcopy=hg)
    h = hs.float().requires_grad_(True)
    gf = g.float().requires_grad_(True)
    bf = b.float().requires_grad_(True)
    torch.nn.functional.layer_norm(h, (D,), gf, bf, 1e-12).backward(dout.float())
    # dx: within the h-copy backward's own bf16 error
    e_got = (got[0].float() - h.grad).abs()
    e_ref = (ref[0].float() - h.grad).abs()
    assert e_got.max().item() <= 2 * e_ref.max().item() + 1e-2 * h.grad.abs().max().item(), (
        e_got.max().item(), e_ref.max().item())
    assert e_got.mean().item() <= 1.5 * e_ref.mean().item() + 1e-4, (e_got.mean().item(), e_ref.mean().item())
    # dgamma / dbeta: sums over 4096 rows of dout x xhat, where the output-based xhat carries
    # out's bf16 rounding (the h copy's rounding is inside the reference): bf16-level agreement
    for k, want in ((2, gf.grad), (3, bf.grad)):
        torch.testing.assert_close(got[k], want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


@pytest.mark.parametrize("R,D", [(2048, 768), (2048, 2048), (70000, 2048), (512, 128)])
def test_add_ln_dropout_statistics_and_consistency(R, D):
    torch.manual_seed(0)
    p = 0.1
    y = torch.ones(R, D, device="cuda").bfloat16()
    g = torch.ones(D, device="cuda").bfloat16()
    b = torch.zeros(D, device="cuda").bfloat16()
    out, hs, mean, rstd = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 3)
    kept = (hs.float() != 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01
    # same seed/offset -> same mask; different offset -> different mask
    _, hs2, _, _ = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 3)
    _, hs3, _, _ = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 4)
    assert torch.equal(hs, hs2) and not torch.equal(hs, hs3)
    # backward regenerates the same mask: dy is zero exactly where dropped
    dout = torch.randn(R, D, device="cuda").bfloat16()
    _, dy, _, _, dyb = _ext().add_ln_bwd(dout, hs, mean, rstd, g, p, 7, 3, False, True, True)
    assert torch.equal(dy == 0, hs == 0)
    torch.testing.assert_close(dyb, dy.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("R,D", [(2048, 768), (8192, 768), (1024, 2048), (32768, 768)])
def test_add_ln_bwd_deferred_partials(R, D):
    """add_ln_bwd(part_buf=...) over three micro-batches (store, add, add) and one
    ln_colreduce give the dgamma / dbeta / colsum(dy) that three immediate calls accumulate."""
    ext = _ext()
    n = ext.ln_bwd_partials(R, D)
    assert n > 0
    torch.manual_seed(0)
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(D, device="cuda")).bfloat16()
    acc_ref = [torch.zeros(D, device="cuda") for _ in range(3)]
    acc_def = [torch.zeros(D, device="cuda") for _ in range(3)]
    part = torch.full((n,), float("nan"), device="cuda")  # stale contents must be overwritten
    for k in range(3):
        y = torch.randn(R, D, device="cuda").bfloat16()
        r = torch.randn(R, D, device="cuda").bfloat16()
        _, hs, mean, rstd = ext.add_ln_fwd(y, r, g, b, 0.1, 1e-12, 5, k)
        dout = torch.randn(R, D, device="cuda").bfloat16()
        d0 = ext.add_ln_bwd(dout, hs, mean, rstd, g, 0.1, 5, k, True, True, True, dg_acc=acc_ref[0],
                            db_acc=acc_ref[1], dyb_acc=acc_ref[2])
        d1 = ext.add_ln_bwd(dout, hs, mean, rstd, g, 0.1, 5, k, True, True, True, dg_acc=acc_def[0],
                            db_acc=acc_def[1], dyb_acc=acc_def[2], part_buf=part, part_acc=k > 0)
        assert torch.equal(d0[0], d1[0]) and torch.equal(d0[1], d1[1])
    assert all(torch.count_nonzero(a).item() == 0 for a in acc_def)  # nothing reduced yet
    ext.ln_colreduce(part, R, D, acc_def[0], acc_def[1], acc_def[2])
    for a, e in zip(acc_def, acc_ref):
        torch.testing.assert_close(a, e, rtol=1e-4, atol=1e-4 * e.abs().max().item())


def test_gemm_nn_dact_kept_bias_partials():
    """gemm_nn_dact(part_out=slot) for two micro-batches, one colsum_acc over both slots ==
    the bias gradient accumulated immediately."""
    ext = _ext()
    torch.manual_seed(0)
    T, N, K = 1024, 256, 1024
    W = (0.05 * torch.randn(N, K, device="cuda")).bfloat16()
    ref = torch.zeros(K, device="cuda")
    got = torch.zeros(K, device="cuda")
    rows = (T // 256) * 2
    buf = torch.empty(2 * rows, K, device="cuda")
    for k in range(2):
        dy = torch.randn(T, N, device="cuda").bfloat16()
        aux = torch.randn(T, K, device="cuda").bfloat16()
        dz0, _ = ext.gemm_nn_dact(dy, W, aux, 1, True, db_acc=ref)
        dz1, db1 = ext.gemm_nn_dact(dy, W, aux, 1, True, db_acc=got, part_out=buf[k * rows:(k + 1) * rows])
        assert db1 is None and torch.equal(dz0, dz1)
    assert torch.count_nonzero(got).item() == 0
    ext.colsum_acc(buf, got)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


@pytest.mark.parametrize("act", ["none", "gelu", "tanh", "silu"])
def test_linear_bias_act_autograd(act):
    torch.manual_seed(0)
    x = torch.randn(333, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.nn.Parameter(torch.randn(512, 256, device="cuda") * 0.05)
    b = torch.nn.Parameter(torch.randn(512, device="cuda") * 0.1)
    y = ops.linear(x, w, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True)
    z = xr @ wr.t() + br
    yr = {"none": z, "gelu": torch.nn.functional.gelu(z), "tanh": torch.tanh(z),
          "silu": torch.nn.functional.silu(z)}[act]
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(w.grad, wr.grad, rtol=3e-2, atol=3e-2 * wr.grad.abs().max().item())
    torch.testing.assert_close(b.grad, br.grad, rtol=3e-2, atol=3e-2 * br.grad.abs().max().item())


def _ln_params(D):
    w = torch.nn.Parameter(1 + 0.1 * torch.randn(D, device="cuda"))
    b = torch.nn.Parameter(0.1 * torch.randn(D, device="cuda"))
    return w, b


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_embed_layernorm_matches_torch(p):
    """DiffuSeq input block dropout(LN(y + pos + temb)) in one kernel vs fp32 torch (the
    dropout mask is read off the kernel's output zeros and applied to the reference)."""
    torch.manual_seed(0)
    B, L, D = 16, 128, 768
    y = torch.randn(B, L, D, device="cuda").bfloat16().requires_grad_(True)
    pos = (0.5 * torch.randn(1, L, D, device="cuda")).bfloat16().requires_grad_(True)
    temb = (0.5 * torch.randn(B, D, device="cuda")).bfloat16().requires_grad_(True)
    w, b = _ln_params(D)
    out = ops.embed_layernorm(y, pos, temb, w, b, p, 1e-12, True)
    keep = (out != 0).float()
    if p > 0:
        assert abs(keep.mean().item() - (1 - p)) < 0.01
    yr, pr, tr = (t.detach().float().requires_grad_(True) for t in (y, pos, temb))
    wr, br = (t.detach().clone().requires_grad_(True) for t in (w, b))
    h = (yr + pr + tr[:, None]).bfloat16().float()  # the kernel rounds h to bf16
    ref = torch.nn.functional.layer_norm(h, (D,), wr, br, 1e-12) * keep / (1 - p)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=3e-2)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g.bfloat16().float())
    torch.testing.assert_close(y.grad.float(), yr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(pos.grad.float(), pr.grad, rtol=2e-2, atol=2e-2 * pr.grad.abs().max().item())
    torch.testing.assert_close(temb.grad.float(), tr.grad, rtol=2e-2, atol=2e-2 * tr.grad.abs().max().item())
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-2, atol=1e-2 * wr.grad.abs().max().item())
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-2, atol=1e-2 * br.grad.abs().max().item())


def test_residual_layernorm_two_outputs():
    """Pre-LN step (x_new, LN(x_new)), x_new = x + h: both outputs carry gradient (the
    kernel adds x_new's own incoming gradient to the LN backward), vs fp32 torch."""
    torch.manual_seed(0)
    B, L, D = 8, 256, 768
    h = torch.randn(B, L, D, device="cuda").bfloat16().requires_grad_(True)
    x = torch.randn(B, L, D, device="cuda").bfloat16().requires_grad_(True)
    w, b = _ln_params(D)
    xn, a = ops.residual_layernorm(h, x, w, b, 0.0, 1e-5, True)
    hr, xr = h.detach().float().requires_grad_(True), x.detach().float().requires_grad_(True)
    wr, br = (t.detach().clone().requires_grad_(True) for t in (w, b))
    xnr = (xr + hr).bfloat16().float()
    xnr.retain_grad()
    ar = torch.nn.functional.layer_norm(xnr, (D,), wr, br, 1e-5)
    torch.testing.assert_close(xn.float(), xnr, rtol=0, atol=0)
    torch.testing.assert_close(a.float(), ar, rtol=2e-2, atol=2e-2)
    ga, gx = torch.randn_like(ar).bfloat16(), torch.randn_like(ar).bfloat16()
    ((a.float() * ga.float()).sum() + (xn.float() * gx.float()).sum()).backward()
    ((ar * ga.float()).sum() + (xnr * gx.float()).sum()).backward()
    torch.testing.assert_close(h.grad.float(), hr.grad, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-2, atol=1e-2 * wr.grad.abs().max().item())


def test_gpt2_input_embedding_dropout_then_ln():
    """GPT-2 input: x = dropout(wte + wpe) (pre-LN dropout of the SUM), a = ln_1(x)."""
    torch.manual_seed(0)
    B, L, D, p = 4, 512, 768, 0.1
    # strictly positive sum, so x == 0 exactly where dropped (the mask is read off x)
    e = (torch.randn(B, L, D, device="cuda").abs() + 0.5).bfloat16().requires_grad_(True)
    pos = (0.1 * torch.rand(1, L, D, device="cuda")).bfloat16()
    w, b = _ln_params(D)
    x, a = ops.residual_layernorm(e, None, w, b, p, 1e-5, True, pos=pos)
    keep = (x != 0).float()
    assert abs(keep.mean().item() - (1 - p)) < 0.01
    ref_x = ((e.float() + pos.float()) * keep / (1 - p)).bfloat16().float()
    torch.testing.assert_close(x.float(), ref_x, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(a.float(), torch.nn.functional.layer_norm(x.float(), (D,), w, b, 1e-5),
                               rtol=2e-2, atol=2e-2)
    x.float().sum().backward()
    torch.testing.assert_close(e.grad.float(), keep / (1 - p), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,L,H", [(64, 128, 768), (5, 64, 128), (17, 256, 256)])
def test_seq_pos_sums_match_torch(B, L, H):
    """csrc/norm.hip seq_pos_sums: both reductions of the input block's gradient in one read."""
    from distributed_pipeline_amd.ops._ext import get_ext
    torch.manual_seed(0)
    d = torch.randn(B * L, H, device="cuda").bfloat16()
    dpos, dtemb = get_ext().seq_pos_sums(d, L, True, True)
    d3 = d.float().view(B, L, H)
    torch.testing.assert_close(dpos, d3.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dtemb, d3.sum(1), rtol=1e-4, atol=1e-3)
    only_t = get_ext().seq_pos_sums(d, L, False, True)
    torch.testing.assert_close(only_t[1], d3.sum(1), rtol=1e-4, atol=1e-3)
