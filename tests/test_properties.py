"""Property tests (hypothesis) for the engine's host-side planning and the settings
round-trip (property tests over shapes / configs)."""
import json

import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from distributed_pipeline_amd.parallel.ddp import plan_buckets
from distributed_pipeline_amd.parallel.flat import FlatParamSpace

_MiB = 1 << 20


@settings(max_examples=40, deadline=None)
@given(sizes=st.lists(st.integers(1, 40000), min_size=1, max_size=24),
       cap_kb=st.integers(4, 400), first_kb=st.integers(1, 200))
def test_bucket_plan_partition(sizes, cap_kb, first_kb):
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    space = FlatParamSpace(params)
    cap, first = cap_kb / 1024, first_kb / 1024
    buckets = plan_buckets(space, cap, first)
    # contiguous cover of the whole (padded) flat buffer, in order
    assert buckets[0][0] == 0 and buckets[-1][1] == space.numel
    assert all(b0[1] == b1[0] and b0[0] < b0[1] for b0, b1 in zip(buckets, buckets[1:]))
    # every parameter in exactly one bucket, and inside its bucket's range
    seen = [id(p) for b in buckets for p in b[2]]
    assert sorted(seen) == sorted(id(p) for p in params)
    for s, e, ps in buckets:
        for p in ps:
            off = space.offsets[id(p)]
            assert s <= off and off + p.numel() <= e
    # a bucket closes as soon as it reaches its limit: dropping its last parameter
    # would leave it under the limit (first bucket: first_mb, then cap_mb) - or early, when
    # the next parameter alone exceeds cap_mb (that one gets a bucket of its own)
    for i, (s, e, ps) in enumerate(buckets[:-1]):
        limit = (first if i == 0 else cap) * _MiB
        last_off = space.offsets[id(ps[-1])]
        assert (last_off - s) * 4 < limit
        nxt = buckets[i + 1][2][0]
        if (e - s) * 4 < limit:
            assert nxt.numel() * 4 > cap * _MiB
    for s, e, ps in buckets:
        if any(p.numel() * 4 > cap * _MiB for p in ps[1:]):
            raise AssertionError("an oversized parameter shares a bucket with earlier ones")
    # the planner the sharded engine uses before the flat space exists agrees
    from distributed_pipeline_amd.parallel.ddp import bucket_members
    idx = {id(p): i for i, p in enumerate(space.layout)}
    assert bucket_members([p.numel() for p in space.layout], cap, first) == [[idx[id(p)] for p in b[2]] for b in buckets]


@settings(max_examples=30, deadline=None)
@given(lr=st.floats(1e-6, 1.0), batch=st.integers(1, 4096), steps=st.integers(0, 10 ** 6),
       ema=st.lists(st.sampled_from(["0.5", "0.9", "0.99", "0.9999"]), min_size=1, max_size=3),
       clip=st.floats(0.0, 10.0), workers=st.integers(0, 8))
def test_settings_json_and_argparse_round_trip(tmp_path_factory, lr, batch, steps, ema, clip, workers):
    from config.train import TrainSettings
    s = TrainSettings(lr=lr, batch_size=batch, learning_steps=steps, ema_rate=",".join(ema),
                      gradient_clipping=clip, data_loader_workers=workers)
    # JSON -> --config_json
    path = tmp_path_factory.mktemp("cfg") / "c.json"
    path.write_text(s.json())
    parser = TrainSettings.to_argparse(add_json=True)
    back = TrainSettings.from_argparse(parser.parse_args(["--config_json", str(path)]))
    assert back == s
    # every field through its CLI flag
    argv = []
    for k, v in json.loads(s.json()).items():
        argv += [f"--{k}", str(v).lower() if isinstance(v, bool) else str(v)]
    back2 = TrainSettings.from_argparse(TrainSettings.to_argparse(add_json=True).parse_args(argv))
    assert back2 == s
