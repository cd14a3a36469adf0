"""bf16 MFMA GEMM kernels (fwd / dgrad / wgrad) vs PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ext():
    from distributed_pipeline_amd.ops._ext import get_ext
    return get_ext(required=True)


@pytest.fixture(params=[256, 128], ids=["tile256", "tile128"])
def tile(request):
    """Run each case on the 256x256 8-phase kernel (where the shape tiles) and on
    the 128x128 kernel."""
    _ext().set_gemm256(request.param == 256)
    yield request.param
    _ext().set_gemm256(True)


def _close(a, r, tol=2e-2):
    err = (a.float() - r).abs().max().item()
    assert err <= tol * max(r.abs().max().item(), 1e-3), (err, r.abs().max().item())


@pytest.mark.parametrize("T,K,N,act", [(256, 128, 128, 0), (512, 768, 2304, 0), (384, 768, 3072, 1),
                                       (128, 256, 384, 2), (256, 128, 512, 3), (768, 768, 3072, 1),
                                       (256, 512, 512, 2), (1024, 128, 768, 3), (512, 3072, 768, 0)])
def test_gemm_nt_bias_act(T, K, N, act, tile):
    torch.manual_seed(0)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    y, z, _ = _ext().gemm_nt(x, W, b, act)
    zr = x.float() @ W.float().t() + b.float()
    yr = {0: zr, 1: torch.nn.functional.gelu(zr), 2: torch.tanh(zr), 3: torch.nn.functional.silu(zr)}[act]
    _close(y, yr)
    if z is not None:
        _close(z, zr)


@pytest.mark.parametrize("T,N,K", [(256, 128, 128), (512, 2304, 768), (384, 768, 3072),
                                   (768, 768, 3072), (512, 3072, 768), (256, 128, 256)])
def test_gemm_nn_dgrad(T, N, K, tile):
    torch.manual_seed(0)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    _close(_ext().gemm_nn(dy, W), dy.float() @ W.float())


@pytest.mark.parametrize("T,N,K", [(128, 128, 128), (4096, 768, 768), (8192, 2304, 768), (1024, 768, 3072),
                                   (640, 256, 256), (256, 512, 768), (32768, 768, 3072),
                                   # a 128-wide side: zero-padded onto the 256 x 256 split-K kernel
                                   (32768, 768, 128), (8192, 128, 768), (512, 384, 128)])
def test_gemm_wgrad_accumulates(T, N, K, tile):
    torch.manual_seed(0)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    dW = torch.randn(N, K, device="cuda")
    db = torch.randn(N, device="cuda")
    ref = dW + dy.float().t() @ x.float()
    refb = db + dy.float().sum(0)
    _ext().gemm_wgrad(dy, x, dW, db)
    _close(dW, ref, 1e-3)
    _close(db, refb, 1e-3)


@pytest.mark.parametrize("nseg", [2, 3, 4, 8])
@pytest.mark.parametrize("T,N,K", [(8192, 768, 768), (8192, 2304, 768), (2048, 768, 3072), (256, 256, 512)])
def test_gemm_wgrad_multi_segment(T, N, K, nseg):
    """One multi-segment split-K launch == the sum of per-segment weight gradients."""
    torch.manual_seed(0)
    dys = [torch.randn(T, N, device="cuda").bfloat16() for _ in range(nseg)]
    xs = [torch.randn(T, K, device="cuda").bfloat16() for _ in range(nseg)]
    dW = torch.randn(N, K, device="cuda")
    db = torch.randn(N, device="cuda")
    ref = dW.clone()
    refb = db.clone()
    for dy, x in zip(dys, xs):
        ref += dy.float().t() @ x.float()
        refb += dy.float().sum(0)
    assert _ext().gemm_wgrad_multi(dys, xs, dW, db)
    _close(dW, ref, 1e-3)
    _close(db, refb, 1e-3)


@pytest.mark.parametrize("T,N,K,act", [(512, 768, 3072, 1), (256, 768, 768, 2), (512, 512, 256, 3)])
def test_gemm_nn_dact(T, N, K, act):
    """dz = (dy W) * act'(aux) with the activation backward fused into the epilogue."""
    torch.manual_seed(0)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    z = torch.randn(T, K, device="cuda").bfloat16()
    zf = z.float()
    if act == 1:
        d = 0.5 * (1 + torch.erf(zf / 2 ** 0.5)) + zf * torch.exp(-0.5 * zf * zf) / (2 * torch.pi) ** 0.5
        aux = z
    elif act == 2:
        aux = torch.tanh(zf).bfloat16()
        d = 1 - aux.float() ** 2
    else:
        s = torch.sigmoid(zf)
        d = s * (1 + zf * (1 - s))
        aux = z
    ref = (dy.float() @ W.float()).bfloat16().float() * d
    dz, db = _ext().gemm_nn_dact(dy, W, aux, act, False)
    _close(dz, ref)
    assert db is None
    dz, db = _ext().gemm_nn_dact(dy, W, aux, act, True)
    _close(dz, ref)
    if db is not None:  # the persistent kernel's fused bias gradient (T % 256 == 0)
        _close(db, dz.float().sum(0), 1e-3)


# Persistent-kernel coverage: many tiles per workgroup (the cross-tile pipeline and its
# in-flight epilogue accounting), K = 128 (one K-iteration per tile), every epilogue.
@pytest.mark.parametrize("T,K,N,act", [(32768, 768, 3072, 1), (65536, 768, 768, 0), (131072, 128, 768, 2),
                                       (16384, 3072, 768, 0), (32768, 768, 2304, 3)])
def test_gemm_persistent_forward_many_tiles(T, K, N, act):
    torch.manual_seed(1)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    y, z, _ = _ext().gemm_nt(x, W, b, act)
    zr = (x.float() @ W.float().t() + b.float()).bfloat16().float()
    yr = {0: zr, 1: torch.nn.functional.gelu(zr), 2: torch.tanh(zr), 3: torch.nn.functional.silu(zr)}[act]
    _close(y, yr)
    if z is not None:
        _close(z, zr)


@pytest.mark.parametrize("T,N,K,act", [(32768, 768, 3072, 1), (65536, 768, 768, 2), (16384, 3072, 768, 3),
                                       (65536, 128, 768, 1)])
def test_gemm_persistent_dgrad_dact_db_many_tiles(T, N, K, act):
    torch.manual_seed(2)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    aux = torch.randn(T, K, device="cuda").bfloat16()
    a = aux.float()
    if act == 1:
        d = 0.5 * (1 + torch.erf(a / 2 ** 0.5)) + a * torch.exp(-0.5 * a * a) / (2 * torch.pi) ** 0.5
    elif act == 2:
        d = 1 - a * a
    else:
        s = torch.sigmoid(a)
        d = s * (1 + a * (1 - s))
    ref = (dy.float() @ W.float()).bfloat16().float() * d
    dz, db = _ext().gemm_nn_dact(dy, W, aux, act, True)
    _close(dz, ref)
    _close(db, dz.float().sum(0), 1e-3)
    dx = _ext().gemm_nn(dy, W)
    _close(dx, dy.float() @ W.float())


@pytest.mark.parametrize("T,N,K", [(65536, 768, 768), (32768, 3072, 768), (512, 2304, 768)])
def test_gemm_nn_accumulate_in_place(T, N, K):
    """dx += dy W (the residual-branch gradient accumulated by the dgrad GEMM epilogue)."""
    torch.manual_seed(3)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    dx = torch.randn(T, K, device="cuda").bfloat16()
    ref = dx.float() + (dy.float() @ W.float()).bfloat16().float()
    assert _ext().gemm_nn_acc_(dy, W, dx)
    _close(dx, ref)


def test_fused_mlp_matches_reference():
    """ops.mlp (fused dgrad+act backward) vs two fp32 Linear layers."""
    from distributed_pipeline_amd.models.layers import MLP
    torch.manual_seed(0)
    for act in ("gelu", "tanh", "silu"):
        m = MLP(256, 1024, 256, act, init_std=0.05).cuda()
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        x = torch.randn(4, 128, 256, device="cuda", requires_grad=True)
        y = m(x.bfloat16())
        g = torch.randn_like(y)
        y.backward(g)
        grads = [p.grad.clone() for p in m.parameters()]
        xg = x.grad.clone()
        for p in m.parameters():
            p.grad = None
        x.grad = None
        yr = m[2](m[0](x))  # fp32 reference path
        yr.backward(g.float())
        _close(y, yr.detach())
        _close(xg, x.grad)
        for a, p in zip(grads, m.parameters()):
            _close(a, p.grad)


@pytest.mark.parametrize("B", [64, 1, 200])
def test_small_token_count_padded_to_native(B):
    """The time-embedding MLP at the reference micro-batch (B = 64 rows of 128) and a Linear
    at odd small row counts run on the native GEMMs with zero-padded rows (no hipBLASLt):
    outputs, input gradients and parameter gradients equal the fp32 reference."""
    from distributed_pipeline_amd.models.layers import MLP, Linear
    from distributed_pipeline_amd.ops import nn as nn_ops
    torch.manual_seed(1)
    m = MLP(128, 512, 768, "silu", init_std=0.05).cuda()
    lin = Linear(768, 256, act="tanh").cuda()
    for mod in (m, lin):
        for p in mod.parameters():
            p.grad = torch.zeros_like(p)
    x = torch.randn(B, 128, device="cuda", requires_grad=True)
    before = nn_ops.PAD_STATS["padded"]
    y = lin(m(x.bfloat16()))
    assert nn_ops.PAD_STATS["padded"] >= before + 2, "small-T GEMMs did not take the padded native path"
    g = torch.randn_like(y)
    y.backward(g)
    grads = [p.grad.clone() for mod in (m, lin) for p in mod.parameters()]
    xg = x.grad.clone()
    for mod in (m, lin):
        for p in mod.parameters():
            p.grad = None
    x.grad = None
    yr = lin(m(x))  # fp32 reference path
    yr.backward(g.float())
    _close(y, yr.detach())
    _close(xg, x.grad)
    for a, p in zip(grads, [p for mod in (m, lin) for p in mod.parameters()]):
        _close(a, p.grad)


def _dact_ref(a, act):
    if act == 1:
        return 0.5 * (1 + torch.erf(a / 2 ** 0.5)) + a * torch.exp(-0.5 * a * a) / (2 * torch.pi) ** 0.5
    if act == 2:
        return 1 - torch.tanh(a) ** 2
    s = torch.sigmoid(a)
    return s * (1 + a * (1 - s))


@pytest.mark.parametrize("T,K,N,act", [(32768, 768, 3072, 1), (16384, 768, 1024, 3), (768, 768, 3072, 1)])
def test_gemm_forward_saves_activation_derivative(T, K, N, act):
    """want_deriv: the persistent forward epilogue stores act'(pre-activation) next to
    act(pre-activation); backward code 4 then multiplies (dz = (dy W) * z)."""
    torch.manual_seed(3)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    y, g, is_d = _ext().gemm_nt(x, W, b, act, True)
    assert is_d  # these shapes tile for the persistent kernel
    zr = (x.float() @ W.float().t() + b.float()).bfloat16().float()
    yr = {1: torch.nn.functional.gelu(zr), 3: torch.nn.functional.silu(zr)}[act]
    _close(y, yr)
    _close(g, _dact_ref(zr, act))
    # backward with the saved derivative: code 4 in the fused dgrad epilogue
    dy = torch.randn(T, 512, device="cuda").bfloat16()
    W2 = (torch.randn(512, N, device="cuda") * 0.05).bfloat16()
    dz, db = _ext().gemm_nn_dact(dy, W2, g, 4, True)
    ref = (dy.float() @ W2.float()).bfloat16().float() * g.float()
    _close(dz, ref)
    torch.testing.assert_close(db, dz.float().sum(0), rtol=1e-2, atol=1e-2 * db.abs().max().item())


@pytest.fixture
def dynamic_schedule():
    ext = _ext()
    ext.set_gemmp_dynamic(True)
    yield
    ext.set_gemmp_dynamic(False)


@pytest.mark.parametrize("T,K,N,act", [(65536, 768, 3072, 1), (131072, 768, 768, 0), (32768, 3072, 768, 0)])
def test_gemm_persistent_dynamic_schedule(T, K, N, act, dynamic_schedule):
    """Per-XCD tile queues (on for world > 1): every tile computed exactly once, same
    results as the static schedule; repeated launches reuse the zeroed queue buffer."""
    torch.manual_seed(4)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    zr = (x.float() @ W.float().t() + b.float()).bfloat16().float()
    yr = {0: zr, 1: torch.nn.functional.gelu(zr)}[act]
    for _ in range(3):
        y, _, _ = _ext().gemm_nt(x, W, b, act)
        _close(y, yr)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    _close(_ext().gemm_nn(dy, W), dy.float() @ W.float())


@pytest.mark.parametrize("T,N,K", [(8192, 768, 3072), (32768, 3072, 768), (16384, 2304, 768), (8192, 768, 768)])
def test_dgrad_with_transposed_weight_matches(T, N, K):
    """wt = W^T (the transposed bf16 shadow, ops/nn.py shadow_t): the data-gradient GEMMs take the
    row-form operand path and give the same products (plain, residual-accumulating, act' times
    dgrad with bias column sums from u8 codes and from a bf16 act')."""
    torch.manual_seed(8)
    ext = _ext()
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    WT = W.t().contiguous()
    ref = dy.float() @ W.float()
    a, b = ext.gemm_nn(dy, W), ext.gemm_nn(dy, W, wt=WT)
    _close(b, ref)
    assert (a.float() - b.float()).abs().max().item() <= 1e-2 * ref.abs().max().item()
    dx0 = torch.randn(T, K, device="cuda").bfloat16()
    d1, d2 = dx0.clone(), dx0.clone()
    assert ext.gemm_nn_acc_(dy, W, d1) and ext.gemm_nn_acc_(dy, W, d2, wt=WT)
    _close(d2, dx0.float() + ref)
    # act' from the ffn-in forward (u8 codes and bf16), through the dact dgrad with column sums
    x = torch.randn(T, 256, device="cuda").bfloat16()
    W1 = (torch.randn(K, 256, device="cuda") * 0.05).bfloat16()
    _, z8, m8 = ext.gemm_nt(x, W1, None, 1, 2)
    _, zb, mb = ext.gemm_nt(x, W1, None, 1, 1)
    assert m8 == 2 and mb == 1
    for aux, act in ((z8, 5), (zb, 4)):
        r1, db1 = ext.gemm_nn_dact(dy, W, aux, act, True)
        r2, db2 = ext.gemm_nn_dact(dy, W, aux, act, True, wt=WT)
        d = (r1.float() - r2.float()).abs().max().item()
        assert d <= 1e-2 * r1.float().abs().max().item(), d
        torch.testing.assert_close(db2, r2.float().sum(0), rtol=1e-2, atol=1e-2 * db2.abs().max().item())


@pytest.mark.parametrize("four_w", [True, False], ids=["wgrad4w", "8phase"])
@pytest.mark.parametrize("T,N,K", [(256, 256, 256), (4096, 768, 768), (8192, 2304, 768), (16384, 768, 3072),
                                   (65536, 3072, 768), (512, 512, 768)])
def test_gemm_wgrad_no_bias(T, N, K, four_w):
    """dW += dy^T x without an in-kernel bias sum: the one-wave-per-SIMD kernel (csrc/wgrad4w.hip,
    split-K workspace merge, or an in-place add when unsplit) and the 8-phase kernel, against fp32."""
    ext = _ext()
    ext.set_wgrad4w(four_w)
    try:
        torch.manual_seed(1)
        dy = torch.randn(T, N, device="cuda").bfloat16()
        x = torch.randn(T, K, device="cuda").bfloat16()
        dW = torch.randn(N, K, device="cuda")
        ref = dW + dy.float().t() @ x.float()
        ext.gemm_wgrad(dy, x, dW, None)
        _close(dW, ref, 1e-3)
    finally:
        ext.set_wgrad4w(False)  # the library default is restored by the multi-segment test below


@pytest.mark.parametrize("nseg", [2, 8])
@pytest.mark.parametrize("T,N,K", [(8192, 768, 768), (8192, 2304, 768), (2048, 768, 3072)])
def test_gemm_wgrad_multi_segment_no_bias(T, N, K, nseg):
    """Multi-segment launches (the deferred weight gradients of the micro-batch schedule) on wgrad4w."""
    _ext().set_wgrad4w(True)
    torch.manual_seed(2)
    dys = [torch.randn(T, N, device="cuda").bfloat16() for _ in range(nseg)]
    xs = [torch.randn(T, K, device="cuda").bfloat16() for _ in range(nseg)]
    dW = torch.randn(N, K, device="cuda")
    ref = dW.clone()
    for dy, x in zip(dys, xs):
        ref += dy.float().t() @ x.float()
    try:
        assert _ext().gemm_wgrad_multi(dys, xs, dW, None)
    finally:
        _ext().set_wgrad4w(False)
    _close(dW, ref, 1e-3)


@pytest.mark.parametrize("with_bias", [False, True])
def test_gemm_wgrad_grouped(with_bias):
    """One grouped launch over several Linears' deferred segments (csrc/gemm256.hip
    wgrad_group_kernel): each dW (and bias column sum) == its fp32 sum of dy_s^T x_s, added onto
    the existing gradient; sites of different shapes and segment counts in one launch."""
    torch.manual_seed(3)
    shapes = [(256, 768, 768, 3), (256, 2304, 768, 1), (512, 768, 3072, 8), (128, 256, 512, 2)]
    dys, xs, dWs, dbs, refs, refbs = [], [], [], [], [], []
    for T, N, K, nseg in shapes:
        d = [torch.randn(T, N, device="cuda").bfloat16() for _ in range(nseg)]
        x = [torch.randn(T, K, device="cuda").bfloat16() for _ in range(nseg)]
        dW = torch.randn(N, K, device="cuda")
        db = torch.randn(N, device="cuda") if with_bias else None
        ref = dW.clone()
        refb = db.clone() if with_bias else None
        for a, b in zip(d, x):
            ref += a.float().t() @ b.float()
            if with_bias:
                refb += a.float().sum(0)
        dys.append(d); xs.append(x); dWs.append(dW); dbs.append(db); refs.append(ref); refbs.append(refb)
    assert _ext().gemm_wgrad_grouped(dys, xs, dWs, dbs)
    for dW, ref, db, refb in zip(dWs, refs, dbs, refbs):
        _close(dW, ref, 1e-3)
        if with_bias:
            _close(db, refb, 1e-3)


def test_gemm_wgrad_grouped_declines_untileable_and_is_deterministic():
    """A site with a 128-wide side declines the whole group (nothing launched); a valid group
    gives the same bits twice (one writer per element)."""
    torch.manual_seed(4)
    d = [torch.randn(256, 128, device="cuda").bfloat16()]
    x = [torch.randn(256, 768, device="cuda").bfloat16()]
    dW = torch.zeros(128, 768, device="cuda")
    assert not _ext().gemm_wgrad_grouped([d], [x], [dW], [None])
    assert dW.abs().max().item() == 0
    d = [torch.randn(1024, 768, device="cuda").bfloat16() for _ in range(4)]
    x = [torch.randn(1024, 3072, device="cuda").bfloat16() for _ in range(4)]
    outs = []
    for _ in range(2):
        dW = torch.zeros(768, 3072, device="cuda")
        assert _ext().gemm_wgrad_grouped([d], [x], [dW], [None])
        outs.append(dW)
    assert torch.equal(outs[0], outs[1])
