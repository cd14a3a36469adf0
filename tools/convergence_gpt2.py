"""Full-size GPT-2 small numerics (BASELINE config #4): the bf16 native engine (hand-written
kernels, fused executed micro-batch, fp32 master weights) against the fp32 stock-PyTorch
reference engine (one fwd/bwd per micro-batch, torch AdamW) over the same synthetic token
batches.  Writes per-step losses and the head/tail window means; exits 1 if the tail-window
means differ by more than 2% (SURVEY §4.5 criterion).

    python tools/convergence_gpt2.py --steps 200 --out profiles/convergence_gpt2_r2.log
"""
import argparse
import itertools
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def _data(B, L, n=8, V=50257):
    g = torch.Generator().manual_seed(321)
    out = []
    for _ in range(n):
        ids = torch.randint(1000, 9000, (B, L), generator=g)  # a narrow id range: learnable unigram
        out.append({"input_ids": ids, "labels": ids.clone()})
    return out


def _train(precision, engine, tmp, steps, B, mb, L):
    from basic_utils import logger
    from utils.initialization import create_model_from_config, seed_all
    from utils.trainer import LMTrainLoop

    logger.configure(dir=os.path.join(tmp, f"{precision}_{engine}"), format_strs=[])
    seed_all(0)
    model = create_model_from_config(model="gpt2", config_name="gpt2", precision=precision, dropout=0.1,
                                     seq_len=L, vocab_size=50257).cuda()
    loop = LMTrainLoop(model=model, data=itertools.cycle(_data(B, L)), batch_size=B, microbatch=mb, lr=1e-4,
                       ema_rate="0.9999", log_interval=10 ** 9, save_interval=10 ** 9, resume_checkpoint="",
                       learning_steps=0, checkpoint_path=tmp, ddp_engine=engine, precision=precision,
                       exec_microbatch=-1 if engine == "torch" else 0)
    losses = []
    torch.manual_seed(7)
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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--microbatch", type=int, default=16)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp()
    ref = _train("fp32", "torch", tmp, a.steps, a.batch, a.microbatch, a.seq_len)
    nat = _train("bf16", "native", tmp, a.steps, a.batch, a.microbatch, a.seq_len)
    w = min(50, a.steps // 4)
    head_r, tail_r = ref[:20].mean().item(), ref[-w:].mean().item()
    head_n, tail_n = nat[:20].mean().item(), nat[-w:].mean().item()
    rel = abs(tail_n - tail_r) / abs(tail_r)
    lines = [f"# GPT-2 small 124M seq{a.seq_len}, batch {a.batch} ({a.batch // a.microbatch} x {a.microbatch}), "
             f"lr 1e-4, {a.steps} steps, synthetic ids in [1000, 9000)",
             "# step fp32_torch_engine bf16_native_engine"]
    lines += [f"{i} {x:.5f} {y:.5f}" for i, (x, y) in enumerate(zip(ref.tolist(), nat.tolist()))]
    lines.append(f"# head(20) fp32 {head_r:.5f} bf16 {head_n:.5f} | tail({w}) fp32 {tail_r:.5f} "
                 f"bf16 {tail_n:.5f} | rel diff {100 * rel:.2f}%")
    text = "\n".join(lines) + "\n"
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text)
    print(lines[-1], flush=True)
    sys.exit(0 if rel <= 0.02 and torch.isfinite(nat).all() else 1)


if __name__ == "__main__":
    main()
