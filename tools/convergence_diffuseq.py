"""Full-size DiffuSeq-base numerics at any sequence length (BASELINE config #3 at seq 512):
the bf16 native engine (fused executed micro-batch) against the fp32 stock-PyTorch engine
(one fwd/bwd per 64-sample micro-batch under no_sync, torch AdamW) on the same synthetic
batches.  Writes per-step losses; exits 1 if the tail-window means differ by more than 2%.

    python tools/convergence_diffuseq.py --seq-len 512 --batch 128 --steps 200 --out profiles/convergence_seq512_r2.log
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


def _train(precision, engine, tmp, steps, B, L, seed=7):
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
                              data=itertools.cycle(_data(B, L)), batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.5,0.9,0.99", log_interval=10 ** 9, save_interval=10 ** 9,
                              resume_checkpoint="", learning_steps=0, checkpoint_path=tmp,
                              ddp_engine=engine, precision=precision,
                              exec_microbatch=-1 if engine == "torch" else 0)
    losses = []
    torch.manual_seed(seed)
    for i in range(steps):
        loop.run_step(next(loop.data))
        losses.append(float(logger.dumpkvs()["loss"]))
        loop.step += 1
        if i % 20 == 0:
            print(f"[{precision}/{engine}] step {i} loss {losses[-1]:.4f}", file=sys.stderr, flush=True)
    return torch.tensor(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--seed", type=int, default=7, help="init / timestep / dropout seed")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp()
    ref = _train("fp32", "torch", tmp, a.steps, a.batch, a.seq_len, a.seed)
    nat = _train("bf16", "native", tmp, a.steps, a.batch, a.seq_len, a.seed)
    w = min(50, a.steps // 4)
    head_r, tail_r = ref[:20].mean().item(), ref[-w:].mean().item()
    head_n, tail_n = nat[:20].mean().item(), nat[-w:].mean().item()
    rel = abs(tail_n - tail_r) / abs(tail_r)
    lines = [f"# DiffuSeq-base 768x12 seq{a.seq_len}, batch {a.batch} ({a.batch // 64} x 64), lr 1e-4, "
             f"{a.steps} steps, synthetic, seed {a.seed}",
             "# step fp32_torch_engine bf16_native_engine"]
    lines += [f"{i} {x:.5f} {y:.5f}" for i, (x, y) in enumerate(zip(ref.tolist(), nat.tolist()))]
    lines.append(f"# head(20) fp32 {head_r:.5f} bf16 {head_n:.5f} | tail({w}) fp32 {tail_r:.5f} "
                 f"bf16 {tail_n:.5f} | rel diff {100 * rel:.2f}%")
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    print(lines[-1], flush=True)
    sys.exit(0 if rel <= 0.02 and torch.isfinite(nat).all() else 1)


if __name__ == "__main__":
    main()
