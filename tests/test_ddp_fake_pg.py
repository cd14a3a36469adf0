"""DDP-engine plumbing at world size 8 in ONE process on torch's fake process group
(SURVEY §4 item 3): collectives are no-ops, so this checks bucket assignment, launch
order from the grad hooks and the forward-time ``no_sync`` decision without 8 ranks."""
import pytest
import torch
import torch.distributed as dist

fake_pg = pytest.importorskip("torch.testing._internal.distributed.fake_pg")

from distributed_pipeline_amd.parallel.ddp import DDPEngine  # noqa: E402


@pytest.fixture
def fake_world():
    dist.init_process_group("fake", store=fake_pg.FakeStore(), rank=3, world_size=8)
    yield
    dist.destroy_process_group()


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])


@pytest.mark.parametrize("native", ["0", "1"])
def test_fake_pg_world8_bucket_launch_order_and_no_sync(fake_world, monkeypatch, native):
    monkeypatch.setenv("DPA_NATIVE_REDUCER", native)
    eng = DDPEngine(_model(), bucket_cap_mb=0.03, first_bucket_mb=0.01)
    assert eng.world_size == 8 and eng.rank == 3
    # buckets tile the flat gradient buffer contiguously, in order
    assert eng.buckets[0].start == 0 and eng.buckets[-1].end == eng.space.numel
    assert all(a.end == b.start for a, b in zip(eng.buckets, eng.buckets[1:]))
    assert len(eng.buckets) >= 3
    launched = []
    if native == "0":
        orig = eng._launch

        def spy(b):
            launched.append(b.index)
            return orig(b)
        monkeypatch.setattr(eng, "_launch", spy)
    x = torch.randn(16, 64)

    # no_sync: forward under the context -> no collective for that backward
    with eng.no_sync():
        eng(x).square().mean().backward()
    eng.finalize()
    assert launched == []
    g_local = eng.space.grad_flat.clone()

    # synced step: every bucket launched exactly once, in bucket order (from the hooks,
    # before finalize), and the no-op fake all-reduce leaves the accumulated grads alone
    eng(x).square().mean().backward()
    if native == "0":
        assert launched == list(range(len(eng.buckets)))
    else:  # the C++ reducer launched every bucket from the hooks, none left for finalize
        assert eng._native.next_bucket() == eng._native.num_buckets() == len(eng.buckets)
        assert list(eng._native.pending()) == [0] * len(eng.buckets)
    eng.finalize()
    torch.testing.assert_close(eng.space.grad_flat, 2 * g_local)
