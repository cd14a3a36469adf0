"""The flat layout follows the order backward completes gradients (parallel/flat.py layout_order,
DiffuSeq ``grad_ready_order``): the DDP engine launches buckets in layout order, so a parameter
completed late but laid out early would hold every later bucket's all-reduce until the end of the
backward.  DiffuSeq registers ``position_embeddings`` / ``LayerNorm`` after its encoder (as the
original does, for checkpoint parity) but uses them at the input."""
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port

CFG = dict(model="diffuseq", config_name="tiny", hidden_size=64, num_layers=2, num_heads=2,
           intermediate_size=128, vocab_size=500, seq_len=16, hidden_dim=16, hidden_t_dim=16,
           dropout=0.0, precision="fp32")


def test_diffuseq_layout_puts_input_block_after_encoder():
    from distributed_pipeline_amd.models import build_model
    from distributed_pipeline_amd.parallel.flat import layout_order
    m = build_model(**CFG)
    lay = layout_order(m.parameters(), order=m.grad_ready_order())
    pos = {id(p): i for i, p in enumerate(lay)}
    enc = [pos[id(p)] for p in m.input_transformers.parameters()]
    for p in list(m.LayerNorm.parameters()) + list(m.position_embeddings.parameters()):
        assert pos[id(p)] > max(enc)
    assert pos[id(m.word_embedding.weight)] == len(lay) - 1
    assert len(lay) == len({id(p) for p in m.parameters()})


def _worker(rank, port, q, native=True, warm=False):
    import os
    import warnings
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if not native:
        os.environ["DPA_NATIVE_REDUCER"] = "0"  # the Python bucket path (GPU tensors over gloo take it)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        torch.manual_seed(0)
        model = build_model(**CFG)
        eng = DDPEngine(model, bucket_cap_mb=0.05, first_bucket_mb=0.02)
        if warm:
            eng.warmup_comm()  # reduces every bucket with no backward: must not spend the first-step check
        diff = create_gaussian_diffusion(steps=50)
        ids = torch.randint(10, 500, (4, 16))
        mask = torch.ones_like(ids)
        mask[:, :4] = 0
        t = torch.randint(0, 50, (4,))
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            terms = diff.training_losses(eng, None, t, dict(input_ids=ids, input_mask=mask))
            terms["loss"].mean().backward()
            eng.finalize()
        bad = [str(w.message)[:200] for w in caught if "DDPEngine" in str(w.message)]
        q.put((rank, len(eng.buckets), eng.bucket_order_report, bad))
    finally:
        dist.destroy_process_group()


import pytest  # noqa: E402


@pytest.mark.parametrize("native,warm", [(True, False), (False, True)])
def test_buckets_complete_in_launch_order_gloo(native, warm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q, native, warm)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _rank, nb, rep, bad in res:
        assert nb >= 4
        assert rep is not None and rep["held_back_by"] == [], rep
        assert not bad, bad
