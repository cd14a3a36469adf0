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
    y, z = _ext().gemm_nt(x, W, b, act)
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
                                   (640, 256, 256), (256, 512, 768), (32768, 768, 3072)])
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
    _close(_ext().gemm_nn_dact(dy, W, aux, act), ref)


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
