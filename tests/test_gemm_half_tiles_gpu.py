"""128-row tiles of the persistent GEMM (gemm256.hip, HMT): the small-T launches of the reference
schedule run twice the tiles.  Every epilogue must give the SAME bits as the 256-row tiles (each
output element sees the same K-order accumulation and the same epilogue math), with the static
and the dynamic tile schedule, and the u8 act' codes written by one tile height must decode the
same when the other reads them."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ext():
    from distributed_pipeline_amd.ops._ext import get_ext
    return get_ext(required=True)


def _modes(fn):
    """fn() under 256-row tiles (mode 0) and forced 128-row tiles (mode 2)."""
    ext = _ext()
    out = []
    try:
        for m in (0, 2):
            ext.set_gemmp_half(m)
            out.append(fn())
    finally:
        ext.set_gemmp_half(-1)
    return out


def _same(a, b):
    for x, y in zip(a if isinstance(a, (tuple, list)) else [a], b if isinstance(b, (tuple, list)) else [b]):
        if isinstance(x, torch.Tensor):
            assert torch.equal(x, y), (x.float() - y.float()).abs().max().item()
        else:
            assert x == y


@pytest.fixture(params=[False, True], ids=["static", "dynamic"])
def schedule(request):
    ext = _ext()
    ext.set_gemmp_dynamic(request.param)
    yield request.param
    ext.set_gemmp_dynamic(False)


@pytest.mark.parametrize("T,K,N,act", [(8192, 768, 3072, 1), (8192, 3072, 768, 0), (8192, 768, 2304, 3),
                                       (32768, 768, 768, 2), (768, 768, 3072, 1)])
@pytest.mark.parametrize("want", [0, 1, 2])
def test_forward_epilogues_bitwise_equal(T, K, N, act, want, schedule):
    torch.manual_seed(0)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    if act == 0 and want:
        pytest.skip("no activation derivative without an activation")
    full, half = _modes(lambda: _ext().gemm_nt(x, W, b, act, want))
    _same(full, half)
    zr = (x.float() @ W.float().t() + b.float()).bfloat16().float()
    yr = {0: zr, 1: torch.nn.functional.gelu(zr), 2: torch.tanh(zr), 3: torch.nn.functional.silu(zr)}[act]
    err = (half[0].float() - yr).abs().max().item()
    assert err <= 2e-2 * yr.abs().max().item()


@pytest.mark.parametrize("T,N,K", [(8192, 768, 3072), (8192, 3072, 768), (8192, 768, 768), (16384, 2304, 768)])
def test_dgrad_epilogues_bitwise_equal(T, N, K, schedule):
    torch.manual_seed(1)
    ext = _ext()
    dy = torch.randn(T, N, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    aux = torch.randn(T, K, device="cuda").bfloat16()
    dx0 = torch.randn(T, K, device="cuda").bfloat16()
    _same(*_modes(lambda: ext.gemm_nn(dy, W)))
    for act in (1, 2, 3, 4):  # EPI 3 (no column sums)
        _same(*_modes(lambda: ext.gemm_nn_dact(dy, W, aux, act, False)[0]))

    def acc():
        d = dx0.clone()
        assert ext.gemm_nn_acc_(dy, W, d)
        return d
    full, half = _modes(acc)
    _same(full, half)
    ref = dx0.float() + (dy.float() @ W.float()).bfloat16().float()
    assert (half.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("T,K,N", [(8192, 768, 3072), (16384, 768, 1024)])
def test_q8_codes_cross_tile_heights(T, K, N):
    """u8 act' codes (tile-native layout) written with 128-row tiles are read by the 256-row
    dgrad (EPI 4, column sums) and vice versa: identical codes, identical gradients."""
    torch.manual_seed(2)
    ext = _ext()
    x = torch.randn(T, K, device="cuda").bfloat16()
    W1 = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b1 = torch.randn(N, device="cuda").bfloat16()
    (yf, z8f, mf), (yh, z8h, mh) = _modes(lambda: ext.gemm_nt(x, W1, b1, 1, 2))
    assert mf == mh == 2
    assert torch.equal(z8f, z8h) and torch.equal(yf, yh)
    dy = torch.randn(T, 512, device="cuda").bfloat16()
    W2 = (torch.randn(512, N, device="cuda") * 0.05).bfloat16()
    full, half = _modes(lambda: ext.gemm_nn_dact(dy, W2, z8h, 5, False)[0])  # EPI 3, ACT 5
    _same(full, half)
    dz4, db4 = ext.gemm_nn_dact(dy, W2, z8h, 5, True)  # EPI 4: always 256-row tiles
    assert torch.equal(dz4, full)
    from distributed_pipeline_amd.ops.nn import act_q8_decode
    ref = (dy.float() @ W2.float()).bfloat16().float() * act_q8_decode(z8h, T, N)
    assert (half.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("T,K,N", [(8192, 768, 768), (8192, 3072, 768)])
def test_residual_dropout_epilogue_bitwise_equal(T, K, N, schedule):
    torch.manual_seed(3)
    ext = _ext()
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(T, N, device="cuda").bfloat16()
    full, half = _modes(lambda: ext.gemm_nt_res(x, W, b, res, 0.1, 1234, 56))
    assert full is not None
    _same(full, half)
