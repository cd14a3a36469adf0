"""The reference 32 x 64 schedule of the headline config with / without the simulated data plane
(parallel/ddp.py enable_sim_comm), for kernel-level comparison under rocprofv3:

    python tools/probes/ref_sim_probe.py --sim 0|1 [--steps 3]

Builds the bench's trainer (synthetic DiffuSeq-base, 2048 x 128 per step, micro-batch 64), runs 3
warmup steps of the micro-batch schedule (plus 2 after enabling the simulated plane), then --steps
timed steps, and prints their wall ms/step."""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sim", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--spec", default="8,1000000,64,0")
    ap.add_argument("--comm", default="high", choices=["high", "normal", "nll"],
                    help="stream of the stand-in kernels: a new highest-priority one, a new normal one, "
                         "or the stream plan's nll stream")
    a = ap.parse_args()
    import torch

    from basic_utils import logger
    from data import load_data_from_args
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop
    logger.configure(dir="/tmp/dpa_ref_sim", format_strs=[])
    seed_all(102)
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="bert-base-uncased",
                                     seq_len=128, vocab_size=30522, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    data = load_data_from_args("train", "synthetic", 2048, deterministic=False, loop=True, num_loader_proc=2,
                               dataset="synthetic", seq_len=128, vocab_size=30522, seed=102, model="diffuseq")
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000, noise_schedule="sqrt")
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model, data=data,
                              batch_size=2048, microbatch=64, lr=1e-4, ema_rate="0.5,0.9,0.99", log_interval=20,
                              save_interval=10 ** 9, resume_checkpoint="", weight_decay=0.0,
                              learning_steps=320000, checkpoint_path="/tmp/dpa_ref_sim", ddp_engine="native",
                              precision="bf16", exec_microbatch=-1)

    def step():
        loop.run_step(next(loop.data))
        if loop.step % loop.log_interval == 0:
            logger.dumpkvs()
        loop.step += 1

    for _ in range(3):
        step()
    if a.sim:
        w, bw, cus, lat = (float(x) for x in a.spec.split(","))
        cs = None
        if a.comm == "normal":
            cs = torch.cuda.Stream()
        elif a.comm == "nll":
            from distributed_pipeline_amd.runtime.streams import plan_stream
            cs = plan_stream(torch.device("cuda", 0), "nll")
        loop.ddp_model.enable_sim_comm(int(w), bw, cus=int(cus), lat_us=lat, comm_stream=cs)
        loop.use_ddp = True
        for _ in range(2):
            step()
    # host time inside the engine's calls (wrapped; the engine's own work, not the model's)
    eng = loop.ddp_model
    acc = {}

    def wrap(obj, name, label=None):
        fn = getattr(obj, name)

        def w(*args, **kw):
            t0 = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                k = label or name
                acc[k] = acc.get(k, 0.0) + time.perf_counter() - t0
        setattr(obj, name, w)

    for n in ("arm_for_backward", "finalize", "_install_hooks", "_remove_hooks", "_arm", "wait_shadow"):
        wrap(eng, n)
    if eng._native is not None:
        nat = eng._native

        class W:
            def __getattr__(self, k):
                return getattr(nat, k)
        wn = W()
        for n in ("disarm", "armed", "mark_ready", "finalize", "arm"):
            f0 = getattr(nat, n)

            def mk(f0=f0, n=n):
                def g(*args):
                    t0 = time.perf_counter()
                    try:
                        return f0(*args)
                    finally:
                        acc["native." + n] = acc.get("native." + n, 0.0) + time.perf_counter() - t0
                return g
            setattr(wn, n, mk())
        eng._native = wn
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    host = time.perf_counter() - t
    torch.cuda.synchronize()
    print(f"sim={a.sim} comm={a.comm}: {(time.perf_counter() - t) / a.steps * 1e3:.2f} ms/step (host enqueue "
          f"{host / a.steps * 1e3:.2f} ms/step); engine host ms/step: "
          + ", ".join(f"{k} {v / a.steps * 1e3:.2f}" for k, v in sorted(acc.items())), flush=True)
    from distributed_pipeline_amd.ops.nn import WGRAD_DEFER
    print("weight-gradient deferral:", WGRAD_DEFER.stats, flush=True)


if __name__ == "__main__":
    main()
