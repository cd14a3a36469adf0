"""CPU semantics of the reference-schedule weight-gradient deferral (ops/nn.py
_WgradDeferral) against a torch stand-in for the extension: operands are held while
``active``, run as one multi-segment call once ``depth`` segments are held, the last
(inactive) backward runs its own segment immediately, ``flush`` runs the rest, and the
accumulated gradient equals the per-micro-batch sum."""
import torch

from distributed_pipeline_amd.ops import nn as nn_ops


class _FakeExt:
    def __init__(self):
        self.calls = []

    def gemm_wgrad(self, dz, x2, gw, gb):
        self.calls.append(1)
        gw += dz.float().t() @ x2.float()
        if gb is not None:
            gb += dz.float().sum(0)

    def gemm_wgrad_multi(self, dzs, xs, gw, gb):
        self.calls.append(len(dzs))
        for dz, x2 in zip(dzs, xs):
            gw += dz.float().t() @ x2.float()
            if gb is not None:
                gb += dz.float().sum(0)
        return True


def _param(shape):
    p = torch.nn.Parameter(torch.zeros(shape))
    p.grad = torch.zeros(shape)
    return p


def test_deferral_pairs_flushes_and_matches(monkeypatch):
    fake = _FakeExt()
    monkeypatch.setattr(nn_ops, "get_ext", lambda *a, **k: fake)
    d = nn_ops._WgradDeferral()
    d.depth = 2
    w, b = _param((8, 4)), _param((8,))
    ref_w, ref_b = torch.zeros(8, 4), torch.zeros(8)
    g = torch.Generator().manual_seed(0)
    for k in range(5):  # micro-batches 0..3 deferred, 4 is the last (armed) one
        dz = torch.randn(16, 8, generator=g).bfloat16()
        x2 = torch.randn(16, 4, generator=g).bfloat16()
        ref_w += dz.float().t() @ x2.float()
        ref_b += dz.float().sum(0)
        last = k == 4
        if last:
            d.active = False
            d.flush()
        else:
            d.active = True
        assert d.offer(w, dz, x2, b, w.grad, b.grad)
        if d.active:
            d.end_backward()  # the trainer's call after every deferred backward
    assert fake.calls == [2, 2, 1], fake.calls
    assert not d.pending
    torch.testing.assert_close(w.grad, ref_w)
    torch.testing.assert_close(b.grad, ref_b)


def test_deferral_flush_runs_odd_tail_and_drop_forgets(monkeypatch):
    fake = _FakeExt()
    monkeypatch.setattr(nn_ops, "get_ext", lambda *a, **k: fake)
    d = nn_ops._WgradDeferral()
    d.depth = 4
    w = _param((8, 4))
    d.active = True
    for _ in range(3):
        assert d.offer(w, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w.grad, None)
    assert fake.calls == [] and len(d.pending[id(w)][2]) == 3
    d.flush()
    assert fake.calls == [3]
    torch.testing.assert_close(w.grad, torch.full((8, 4), 48.0))
    d.offer(w, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w.grad, None)
    d.drop()
    assert not d.pending and not d.active


def test_deferral_off_or_unowned_grads_are_not_taken(monkeypatch):
    fake = _FakeExt()
    monkeypatch.setattr(nn_ops, "get_ext", lambda *a, **k: fake)
    d = nn_ops._WgradDeferral()
    w = _param((8, 4))
    d.active = True
    assert not d.offer(w, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w.grad, None)
    d.depth = 2
    other = torch.zeros(8, 4)  # not p.grad: the caller needs the gradient returned
    assert not d.offer(w, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, other, None)
    assert fake.calls == [] and not d.pending


def test_deferral_respects_the_memory_budget(monkeypatch):
    fake = _FakeExt()
    monkeypatch.setattr(nn_ops, "get_ext", lambda *a, **k: fake)
    d = nn_ops._WgradDeferral()
    d.depth = 4
    d.budget_bytes = 16 * 8 * 2 + 16 * 4 * 2  # room for exactly one held (dz, x2) pair
    w1, w2 = _param((8, 4)), _param((8, 4))
    d.active = True
    assert d.offer(w1, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w1.grad, None)
    assert d.held_bytes == d.budget_bytes and fake.calls == []
    # over budget: w2's gradient runs immediately instead of being held
    assert d.offer(w2, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w2.grad, None)
    assert fake.calls == [1] and id(w2) not in d.pending
    # w1's second segment would need twice the budget: both run now as one launch
    assert d.offer(w1, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w1.grad, None)
    assert fake.calls == [1, 2] and d.held_bytes == 0 and not d.pending


def test_grouped_flush_collects_complete_sites_once_per_weight(monkeypatch):
    """Sites that complete their segments wait in ``ready`` until end_backward(); a weight that
    completed twice before it (no end_backward between) is never put in one grouped launch twice."""
    fake = _FakeExt()
    monkeypatch.setattr(nn_ops, "get_ext", lambda *a, **k: fake)
    d = nn_ops._WgradDeferral()
    d.depth = 2
    w = _param((8, 4))
    d.active = True
    for _ in range(4):
        assert d.offer(w, torch.ones(16, 8).bfloat16(), torch.ones(16, 4).bfloat16(), None, w.grad, None)
    assert fake.calls == [] and len(d.ready) == 2 and not d.pending
    d.end_backward()  # CPU tensors: not groupable, one multi-segment call per entry
    assert fake.calls == [2, 2] and not d.ready and d.held_bytes == 0
    torch.testing.assert_close(w.grad, torch.full((8, 4), 64.0))
