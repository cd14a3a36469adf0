"""Sort-free id orderings (csrc/sort.hip): the STABLE counting sort behind the embedding gradients
and the stable 0/1 partition behind the logged nll, against torch references.  The embedding
gradient over the counting sort is compared with an fp64 ``index_add_`` on duplicate-heavy ids
(a few hot ids holding most tokens, as padding does in real data), and two runs of it must give
bitwise-equal gradients (one writer per row, a fixed summation order)."""
import pytest
import torch

from distributed_pipeline_amd.ops._ext import get_ext

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _check_bucket_sort(ids, V):
    s, p = get_ext().id_sort(ids, V)
    flat = ids.reshape(-1)
    n = flat.numel()
    assert s.shape == (n,) and p.shape == (n,)
    # p is a permutation and s = ids[p]
    assert torch.equal(torch.sort(p).values, torch.arange(n, device=DEV))
    assert torch.equal(s, flat[p])
    # buckets ascending, out-of-range ids (bucket V) last, and STABLE: inside a bucket the
    # tokens keep their index order (the permutation torch's stable argsort gives)
    b = torch.where((s >= 0) & (s < V), s, torch.full_like(s, V))
    assert bool((b[1:] >= b[:-1]).all())
    key = torch.where((flat >= 0) & (flat < V), flat, torch.full_like(flat, V))
    assert torch.equal(p, torch.argsort(key, stable=True))
    return s, p


@pytest.mark.parametrize("n,V", [(262144, 30522), (1000, 7), (4097, 50257), (64, 1)])
def test_id_sort_uniform(n, V):
    g = torch.Generator(device="cpu").manual_seed(n)
    ids = torch.randint(0, V, (n,), generator=g).to(DEV)
    _check_bucket_sort(ids, V)


def test_id_sort_duplicate_heavy_and_out_of_range():
    g = torch.Generator(device="cpu").manual_seed(1)
    n, V = 200003, 30522
    ids = torch.randint(0, V, (n,), generator=g)
    hot = torch.rand(n, generator=g)
    ids[hot < 0.5] = 0          # a padding-like id on half the tokens
    ids[(hot >= 0.5) & (hot < 0.6)] = 102
    ids[(hot >= 0.6) & (hot < 0.62)] = -100   # ignored
    ids[(hot >= 0.62) & (hot < 0.63)] = V + 5  # out of range
    _check_bucket_sort(ids.to(DEV), V)


@pytest.mark.parametrize("n", [262144, 1, 1000, 5000])
def test_partition01_is_stable_argsort(n):
    g = torch.Generator(device="cpu").manual_seed(n)
    m = (torch.rand(n, generator=g) > 0.45).long().to(DEV)
    m[::7] *= 3  # any nonzero counts as one
    order = get_ext().partition01(m)
    ref = torch.argsort((m != 0).long(), descending=True, stable=True)
    assert torch.equal(order, ref)


@pytest.mark.parametrize("E", [128, 768])
def test_emb_grad_matches_index_add_duplicate_heavy(E):
    g = torch.Generator(device="cpu").manual_seed(E)
    V, n = 30522, 65536
    ids = torch.randint(0, V, (n,), generator=g)
    ids[torch.rand(n, generator=g) < 0.4] = 3
    ids = ids.to(DEV)
    dy = torch.randn(n, E, generator=g).to(DEV).to(torch.bfloat16)
    dW = torch.zeros(V, E, device=DEV)
    get_ext().emb_grad(ids, dy, dW)
    ref = torch.zeros(V, E, dtype=torch.float64, device=DEV).index_add_(0, ids, dy.double())
    err = (dW.double() - ref).abs().max().item()
    assert err <= 3e-5 * max(1.0, ref.abs().max().item()), err


def test_emb_qsample_bwd_uses_counting_sort_same_result():
    """The fused q_sample backward (counting-sort path, E = 128) against an fp64 index_add_."""
    g = torch.Generator(device="cpu").manual_seed(5)
    B, L, E, V = 64, 128, 128, 30522
    ids = torch.randint(0, V, (B, L), generator=g)
    ids[:, 100:] = 0
    ids = ids.to(DEV)
    mask = (torch.rand(B, L, generator=g) > 0.3).long().to(DEV)
    t = torch.randint(0, 2000, (B,), generator=g).to(DEV)
    sa = torch.rand(2000, generator=g).to(DEV)
    d_xs = torch.randn(B, L, E, generator=g).to(DEV)
    d_xt = torch.randn(B, L, E, generator=g).to(DEV).to(torch.bfloat16)
    dW = torch.zeros(V, E, device=DEV)
    get_ext().emb_qsample_bwd(ids, mask, t, sa, d_xs, None, d_xt, dW)
    a = torch.where(mask != 0, sa[t][:, None].expand(B, L), torch.ones(B, L, device=DEV))
    rows = d_xs.double() + a[..., None].double() * d_xt.double()
    ref = torch.zeros(V, E, dtype=torch.float64, device=DEV).index_add_(0, ids.reshape(-1), rows.reshape(-1, E))
    err = (dW.double() - ref).abs().max().item()
    assert err <= 3e-5 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("E,n", [(128, 262144), (768, 65536)])
def test_emb_grad_bitwise_reproducible(E, n):
    """Two runs of the embedding gradient over the same inputs give the same bits (SURVEY 7.4:
    the tied-embedding reduction deterministic), onto a non-zero gradient buffer, including a
    padding-like id whose run crosses thousands of chunk boundaries."""
    g = torch.Generator(device="cpu").manual_seed(11)
    V = 30522
    ids = torch.randint(0, V, (n,), generator=g)
    ids[torch.rand(n, generator=g) < 0.45] = 0
    ids = ids.to(DEV)
    dy = torch.randn(n, E, generator=g).to(DEV).to(torch.bfloat16)
    base = torch.randn(V, E, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        dW = base.clone()
        get_ext().emb_grad(ids, dy, dW)
        outs.append(dW)
    assert torch.equal(outs[0], outs[1])
    ref = base.double().index_add_(0, ids, dy.double())
    err = (outs[0].double() - ref).abs().max().item()
    assert err <= 3e-5 * max(1.0, ref.abs().max().item()), err


def test_emb_qsample_bwd_bitwise_reproducible():
    g = torch.Generator(device="cpu").manual_seed(6)
    B, L, E, V = 2048, 128, 128, 30522
    ids = torch.randint(0, V, (B, L), generator=g)
    ids[:, 90:] = 0
    ids = ids.to(DEV)
    mask = (torch.rand(B, L, generator=g) > 0.3).long().to(DEV)
    t = torch.randint(0, 2000, (B,), generator=g).to(DEV)
    sa = torch.rand(2000, generator=g).to(DEV)
    d_xs = torch.randn(B, L, E, generator=g).to(DEV)
    d_xt = torch.randn(B, L, E, generator=g).to(DEV).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        dW = torch.zeros(V, E, device=DEV)
        get_ext().emb_qsample_bwd(ids, mask, t, sa, d_xs, None, d_xt, dW)
        outs.append(dW)
    assert torch.equal(outs[0], outs[1])
