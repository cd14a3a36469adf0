"""Diagnostics of the simulated data plane (parallel/ddp.py enable_sim_comm): per-bucket host hook
times and device timelines for the fused and the micro-batch schedule of a DiffuSeq-base step.

    python tools/probes/sim_comm_probe.py [--batch 512] [--layers 12]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--exec", type=int, default=0, help="executed micro-batch (0 = whole batch)")
    a = ap.parse_args()
    from basic_utils import logger
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop
    logger.configure(dir="/tmp/dpa_sim_probe", format_strs=[])
    seed_all(0)
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="bert-base-uncased",
                                     num_layers=a.layers, vocab_size=30522, seq_len=128, hidden_dim=128,
                                     hidden_t_dim=128, dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(1)
    B, L = a.batch, 128
    batch = {"input_ids": torch.randint(1000, 30522, (B, L), generator=g),
             "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                      torch.ones(B, L - 48, dtype=torch.long)], 1)}
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter([batch] * 100), batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.9999", log_interval=10 ** 6, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=100, checkpoint_path="/tmp/dpa_sim_probe", ddp_engine="native",
                              precision="bf16", device_prefetch=False, exec_microbatch=a.exec)
    eng = loop.ddp_model
    eng.enable_sim_comm(8, 153.0, cus=64, lat_us=10.0)
    loop.use_ddp = True
    nat = eng._native
    hook_t = []
    orig = nat.mark_ready

    class Wrap:
        def __getattr__(self, k):
            return getattr(nat, k)

        def mark_ready(self, i):
            hook_t.append((time.perf_counter(), i, nat.next_bucket()))
            return orig(i)
    eng._native = Wrap()
    for step in range(3):
        hook_t.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run_step(batch)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        launched = [(round((t - t0) * 1e3, 2), i, nb) for t, i, nb in hook_t]
        firsts = {}
        for t, i, nb in launched:
            firsts.setdefault(nb, t)
        print(json.dumps({"step": step, "host_ms": round(t_host * 1e3, 2), "total_ms": round(t_all * 1e3, 2),
                          "hooks": len(hook_t), "first_hook_ms": launched[0][0] if launched else None,
                          "last_hook_ms": launched[-1][0] if launched else None,
                          "next_bucket_at_hook_ms": firsts,
                          "timeline": eng.sim_timeline(), "stats": eng.sim_stats(reset=True)}), flush=True)


if __name__ == "__main__":
    main()
