"""Direct xGMI IPC all-reduce kernel (csrc/ipc_allreduce.hip).

Single-GPU correctness of the reduction + signalling protocol: W simulated ranks
run in ONE launch (gridDim.y = W, every block acting as its rank with the exact
per-rank code path, peers' buffers being other allocations on the same device).
Repeated calls exercise the epoch counters and both parity halves of the staging
buffer; mixed one-shot / two-shot calls exercise flag-slot reuse across modes.
The multi-process path (hipIpc handle exchange in the reducer) is exercised by
the driver's 8-GPU node only when DPA_IPC_ALLREDUCE=1 (opt-in).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ext():
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    assert hasattr(ext, "ipc_allreduce_sim")
    return ext


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("two_shot", [False, True])
@pytest.mark.parametrize("n", [4, 1000, 65536, 100_000])
def test_ipc_allreduce_sim(W, two_shot, n):
    ext = _ext()
    g = torch.Generator(device="cuda").manual_seed(W * 7 + n)
    xs = [torch.randn(n, device="cuda", generator=g) for _ in range(W)]
    ref = torch.stack(xs).double().sum(0)
    err = ext.ipc_allreduce_sim(xs, int(two_shot), 1)
    assert err == 0
    for x in xs:
        torch.testing.assert_close(x.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("W", [2, 8])
def test_ipc_allreduce_repeated_epochs(W):
    """k calls of an all-reduce on all-ones inputs give W**k (epochs 1..k, both parities;
    mode 2 alternates one-shot and two-shot, whose block counts differ)."""
    ext = _ext()
    n = 40000
    xs = [torch.ones(n, device="cuda") for _ in range(W)]
    for mode in (0, 1, 2):
        for x in xs:
            x.fill_(1.0)
        assert ext.ipc_allreduce_sim(xs, mode, 3) == 0
        for x in xs:
            assert torch.all(x == float(W) ** 3)


def test_ipc_allreduce_rejects_bad_shapes():
    ext = _ext()
    xs = [torch.ones(6, device="cuda") for _ in range(2)]
    with pytest.raises(RuntimeError):
        ext.ipc_allreduce_sim(xs, 0, 1)


@pytest.mark.parametrize("W", [2, 4, 8])
def test_ipc_allreduce_reducer_issue_pattern(W):
    """The BucketReducer's direct-mode sequence (csrc/comm/reducer.cpp launch_direct): buckets of
    different sizes back to back through one staging buffer sized for the largest, the epoch
    advancing per bucket (alternating parity halves bucket to bucket, across steps), one-shot
    below 256 KiB and two-shot above - over 3 steps = 15 consecutive epochs.  All-ones inputs
    make the expected value of every element W ** steps."""
    ext = _ext()
    sizes = [4096, 100_000, 64, 70_000, 24]  # 16 KiB / 400 KB / ... : both modes, odd sizes
    steps = 3
    buckets = [[torch.ones(n, device="cuda") for _ in range(W)] for n in sizes]
    assert ext.ipc_allreduce_sim_buckets(buckets, steps) == 0
    for b in buckets:
        for x in b:
            assert torch.all(x == float(W) ** steps), (x.numel(), x.unique())
    # random data, one step: every bucket equals the fp64 sum of its rank slices
    g = torch.Generator(device="cuda").manual_seed(W)
    buckets = [[torch.randn(n, device="cuda", generator=g) for _ in range(W)] for n in sizes]
    refs = [torch.stack(b).double().sum(0) for b in buckets]
    assert ext.ipc_allreduce_sim_buckets(buckets, 1) == 0
    for b, ref in zip(buckets, refs):
        for x in b:
            torch.testing.assert_close(x.double(), ref, rtol=1e-5, atol=1e-5)
