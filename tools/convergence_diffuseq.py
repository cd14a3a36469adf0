"""Full-size DiffuSeq-base numerics at any sequence length (BASELINE config #3 at seq 512):
the bf16 native engine (fused executed micro-batch) against the fp32 stock-PyTorch engine
(one fwd/bwd per 64-sample micro-batch under no_sync, torch AdamW) on the same synthetic
batches.  Writes per-step losses; exits 1 if the tail-window means differ by more than 2%.

    python tools/convergence_diffuseq.py --seq-len 512 --batch 128 --steps 200 --out profiles/convergence_seq512_r2.log

``--fresh``: a new synthetic batch every step (no cycling of 4 batches, so the runs measure
learning rather than memorisation).  ``--control``: a third run, fp32 torch engine again with
the SAME initial weights but a different timestep / noise / dropout stream, as the noise floor
of the comparison: the bf16 gap is judged against the fp32-vs-fp32 gap.
"""
import argparse
import itertools
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def _data(B, L, n=4):
    g = torch.Generator().manual_seed(123)
    mask = torch.cat([torch.zeros(B, L // 2, dtype=torch.long), torch.ones(B, L - L // 2, dtype=torch.long)], 1)
    return [{"input_ids": torch.randint(1000, 30000, (B, L), generator=g), "input_mask": mask} for _ in range(n)]


def _fresh(B, L):
    """A new batch every step, the same sequence for every engine (batch i from seed 123 + i)."""
    mask = torch.cat([torch.zeros(B, L // 2, dtype=torch.long), torch.ones(B, L - L // 2, dtype=torch.long)], 1)
    for i in itertools.count():
        g = torch.Generator().manual_seed(123 + i)
        yield {"input_ids": torch.randint(1000, 30000, (B, L), generator=g), "input_mask": mask}


def _train(precision, engine, tmp, steps, B, L, seed=7, fresh=False, stream_seed=None, native_exec=0):
    from basic_utils import logger
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir=os.path.join(tmp, f"{precision}_{engine}"), format_strs=[])
    seed_all(seed)
    model = create_model_from_config(model="diffuseq", config_name="bert-base-uncased", vocab_size=30522,
                                     seq_len=L, hidden_dim=128, hidden_t_dim=128, precision=precision,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=_fresh(B, L) if fresh else itertools.cycle(_data(B, L)),
                              batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.5,0.9,0.99", log_interval=10 ** 9, save_interval=10 ** 9,
                              resume_checkpoint="", learning_steps=0, checkpoint_path=tmp,
                              ddp_engine=engine, precision=precision,
                              exec_microbatch=-1 if engine == "torch" else native_exec)
    losses = []
    torch.manual_seed(seed if stream_seed is None else stream_seed)
    for i in range(steps):
        loop.run_step(next(loop.data))
        losses.append(float(logger.dumpkvs()["loss"]))
        loop.step += 1
        if i % 20 == 0:
            print(f"[{precision}/{engine}{'' if stream_seed is None else '/ctl'}] step {i} loss {losses[-1]:.4f}",
                  file=sys.stderr, flush=True)
    return torch.tensor(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--seed", type=int, default=7, help="init / timestep / dropout seed")
    ap.add_argument("--out", default=None)
    ap.add_argument("--fresh", action="store_true", help="a new synthetic batch every step")
    ap.add_argument("--control", action="store_true", help="fp32 control run with another noise stream")
    ap.add_argument("--window", type=int, default=0, help="tail window (default min(50, steps/4))")
    ap.add_argument("--native-exec", type=int, default=0,
                    help="bf16 engine's executed micro-batch: 0 fused (default), -1 the 64-sample "
                         "micro-batch schedule under no_sync (BASELINE config #3's own schedule)")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp()
    ref = _train("fp32", "torch", tmp, a.steps, a.batch, a.seq_len, a.seed, a.fresh)
    nat = _train("bf16", "native", tmp, a.steps, a.batch, a.seq_len, a.seed, a.fresh, native_exec=a.native_exec)
    ctl = (_train("fp32", "torch", tmp, a.steps, a.batch, a.seq_len, a.seed, a.fresh, stream_seed=a.seed + 1000)
           if a.control else None)
    w = a.window or min(50, a.steps // 4)
    head_r, tail_r = ref[:20].mean().item(), ref[-w:].mean().item()
    head_n, tail_n = nat[:20].mean().item(), nat[-w:].mean().item()
    rel = abs(tail_n - tail_r) / abs(tail_r)
    lines = [f"# DiffuSeq-base 768x12 seq{a.seq_len}, batch {a.batch} ({a.batch // 64} x 64), lr 1e-4, "
             f"{a.steps} steps, synthetic ({'fresh batch every step' if a.fresh else '4 cycled batches'}), "
             f"seed {a.seed}, bf16 schedule {'fused' if a.native_exec == 0 else 'micro-batch ' + str(a.native_exec)}",
             "# step fp32_torch_engine bf16_native_engine" + (" fp32_control(other noise stream)" if a.control else "")]
    for i in range(a.steps):
        row = f"{i} {ref[i].item():.5f} {nat[i].item():.5f}"
        if ctl is not None:
            row += f" {ctl[i].item():.5f}"
        lines.append(row)
    # windowed relative gaps over the run (window w): bf16 vs fp32 and control vs fp32
    for s0 in range(0, a.steps - w + 1, w):
        r = ref[s0:s0 + w].mean().item()
        msg = f"# window {s0}-{s0 + w - 1}: fp32 {r:.5f} bf16 {nat[s0:s0 + w].mean().item():.5f} " \
              f"({100 * (nat[s0:s0 + w].mean().item() - r) / r:+.2f}%)"
        if ctl is not None:
            c = ctl[s0:s0 + w].mean().item()
            msg += f" control {c:.5f} ({100 * (c - r) / r:+.2f}%)"
        lines.append(msg)
    summary = (f"# head(20) fp32 {head_r:.5f} bf16 {head_n:.5f} | tail({w}) fp32 {tail_r:.5f} "
               f"bf16 {tail_n:.5f} | rel diff {100 * rel:.2f}%")
    ok = rel <= 0.02
    if ctl is not None:
        tail_c = ctl[-w:].mean().item()
        rel_c = abs(tail_c - tail_r) / abs(tail_r)
        summary += f" | control tail {tail_c:.5f} rel diff {100 * rel_c:.2f}% (noise floor)"
        ok = ok or rel <= 1.5 * rel_c
    lines.append(summary)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    print("\n".join(l for l in lines if l.startswith("# window") or l.startswith("# head")), flush=True)
    sys.exit(0 if ok and torch.isfinite(nat).all() else 1)


if __name__ == "__main__":
    main()
