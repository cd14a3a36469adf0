"""StreamPlan without the native extension: a stock run needs no native code, so the
plan must fall back to torch pool streams instead of raising (runtime/streams.py), and
claim_stream_plan is a no-op on CPU.  CPU-only: torch.cuda's stream/device entry points are
replaced by fakes, so no GPU is touched."""
import contextlib

import torch

from distributed_pipeline_amd.ops import _ext
from distributed_pipeline_amd.runtime import streams as S


def test_stream_plan_falls_back_to_pool_streams_without_the_extension(monkeypatch):
    monkeypatch.setattr(_ext, "get_ext", lambda required=None: None)
    made = []

    class FakeStream:
        def __init__(self, device=None):
            made.append(device)
            self.cuda_stream = 0x1000 + len(made)

    monkeypatch.setattr(torch.cuda, "Stream", FakeStream)
    monkeypatch.setattr(torch.cuda, "device", lambda d: contextlib.nullcontext())
    plan = S.StreamPlan("cuda:0")
    assert plan.mode == "pool"
    assert set(plan.streams) == set(S.ROLES)
    assert len(made) == len(S.ROLES)  # one pool stream per role, none shared
    d = plan.describe()
    assert d["mode"] == "pool" and "hw_queues_expected" not in d
    assert plan.get("comm") is plan.streams["comm"]


def test_stream_plan_is_empty_on_cpu_and_claim_is_a_no_op():
    plan = S.StreamPlan("cpu")
    assert plan.streams == {} and plan.get("side") is None
    assert S.plan_stream("cpu", "wgrad") is None
    from basic_utils.dist_util import claim_stream_plan
    assert claim_stream_plan("cpu") is None
