"""
Headline benchmark (BASELINE.json): DiffuSeq-base, seq 128, DDP training
throughput on N MI355X of one node, one process per GPU over RCCL/xGMI.

    python bench.py --gpus N --steps K --warmup W
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py ...)

A *step* is the reference's optimizer step (reference utils/trainer.py:198-201 +
config/train.py defaults): 2048 samples per rank (global batch 2048*N) made of
micro-batches of 64, one all-reduce, AdamW, 3 EMA rates, grad-norm logging,
linear LR decay, logger dump every 20 steps.  Synthetic tokens, random-init
weights.

Step schedule.  The reference runs one forward/backward per 64-sample
micro-batch (32 per step, no_sync on all but the last).  The headline number uses
this framework's default schedule (``exec_microbatch=0`` = auto): the 32
micro-batches execute as ONE forward/backward over the whole 2048-sample batch,
whose loss is scaled so the gradient equals the reference's sum of per-micro-batch
means (tests/test_trainer.py checks this, also for uneven chunks).  That is the
MI355X-first choice - 288 GB of HBM hold the activations, and 8192-token GEMMs
fill a 256-CU chip only ~60%.  The reference's own 32 x 64 schedule is measured in
the same process and reported under ``reference_schedule`` (``--ref-steps``).

Reported ``value`` is the whole-job aggregate: optimizer steps/s x N
(= samples/s / 2048), so it scales with N under weak scaling; rank-local
steps/s, samples/s and tokens/s are reported alongside.

``--reference-equivalent`` runs the reference's configuration instead (fp32,
torch DistributedDataParallel with bucket_cap_mb=128, torch AdamW, eager
PyTorch model) - the measured baseline in BASELINE.md.  ``--stock`` keeps every op
on stock PyTorch / ATen (hipBLASLt GEMMs, SDPA attention, ATen LayerNorm and CE:
``use_hip_kernels=False``); with ``--reference-equivalent --precision bf16 --stock``
that is the like-for-like bf16 baseline (``vs_stock_bf16``), at the reference's
micro-batch 64 by default or fused with ``--exec-microbatch 0`` (auto).
"""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "train steps/sec (whole node), DiffuSeq-base seq128 DDP at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=2048)
    ap.add_argument("--microbatch", type=int, default=64)
    ap.add_argument("--exec-microbatch", type=int, default=None,
                    help="samples per executed fwd/bwd: 0 = auto (whole batch), -1 = microbatch (reference "
                         "schedule); default auto, or -1 with --reference-equivalent")
    ap.add_argument("--ref-warmup", type=int, default=2,
                    help="untimed reference-schedule steps first (its two extra HIP streams grow their own "
                         "allocator pools in the first steps)")
    ap.add_argument("--ref-steps", type=int, default=8,
                    help="also time this many steps of the reference 32 x 64 schedule (0 = skip)")
    ap.add_argument("--ref-graph", type=int, default=0,
                    help="run the reference schedule as a replayed HIP graph (TrainLoop cuda_graph; 0 = eager: "
                         "the replay measured 249-251 vs 228-229 ms/step eager, profiles/ref_schedule_graph_ab_r4.txt)")
    ap.add_argument("--ref-windows", type=int, default=1,
                    help="time the reference schedule in this many back-to-back windows of --ref-steps "
                         "(the mean over all is reported, each window under windows_ms)")
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--config-name", default="bert-base-uncased")
    ap.add_argument("--model", default="diffuseq")
    ap.add_argument("--reference-equivalent", action="store_true")
    ap.add_argument("--stock", action="store_true",
                    help="stock PyTorch ops only (use_hip_kernels=False): the like-for-like baseline")
    ap.add_argument("--precision", default=None)
    # 0 = measured at startup on the job's process group (parallel/ddp.py tune_bucket_sizes);
    # world 1 has no reduction and keeps 32 / 4
    ap.add_argument("--bucket-cap-mb", type=float, default=0.0)
    ap.add_argument("--first-bucket-mb", type=float, default=0.0)
    ap.add_argument("--zero1", type=int, default=0, help="ZeRO-1 sharded optimizer (N > 1)")
    ap.add_argument("--grad-wire", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--data-workers", type=int, default=2)
    ap.add_argument("--log-interval", type=int, default=20)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--project", default="",
                    help="N = 1 only, after the measurements: a one-GPU PROJECTION of the W > 1 data plane. "
                         "';'-separated specs W,busbw_GBps[,cus[,lat_us[,bucket_cap_mb,first_bucket_mb]]] ('/' "
                         "may replace ','): each "
                         "bucket's all-reduce is replaced by a calibrated kernel on the reducer's comm stream "
                         "(parallel/ddp.py enable_sim_comm); reported under 'projection'")
    ap.add_argument("--project-schedules", default="fused,reference",
                    help="schedules the projection times: fused and/or reference (the 32 x 64 one)")
    ap.add_argument("--project-reps", type=int, default=2,
                    help="alternating plain / simulated segments per projection point (medians reported)")
    ap.add_argument("--project-wire", default="",
                    help="'fp32,bf16': time each spec with both wire formats (default: --grad-wire)")
    ap.add_argument("--comm-probe", type=int, default=1,
                    help="N > 1: after the timed runs, time the full gradient reduction and the "
                         "process group's all-reduce at 1-128 MB (reported under comm_probe)")
    return ap.parse_args()


def topology():
    """xGMI topology of the node (recorded with every measurement):
    `amd-smi topology --json` link types / hop counts between the visible GPUs,
    compacted; None when the tool is unavailable."""
    import subprocess
    try:
        r = subprocess.run(["amd-smi", "topology", "--json"], capture_output=True, text=True, timeout=20)
        data = json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else None
    except Exception:  # noqa: BLE001
        return None
    if not data:
        return None
    rows = data if isinstance(data, list) else data.get("topology", [data])
    out = []
    for row in rows:
        if not isinstance(row, dict):
            continue
        gpu = row.get("gpu")
        links = row.get("links") or []
        kinds = sorted({str(l.get("link_type")) for l in links if isinstance(l, dict) and l.get("link_type")})
        hops = [l.get("num_hops") for l in links if isinstance(l, dict) and "num_hops" in l]
        out.append({"gpu": gpu, "link_types": kinds, "peers": len(links), "max_hops": max(hops) if hops else None})
    return out or None


def comm_probe(loop, engine, dev, sync):
    """After the timed runs (N > 1): the data plane's full gradient reduction
    with this run's bucket plan (``DDPEngine.reduce_all_now``: every bucket, back to back,
    nothing to overlap with - the cost a step hides under its backward) and the process
    group's all-reduce bus bandwidth at bucket sizes 1-128 MB (the data behind the 4 MiB first
    bucket / 32 MiB buckets), and the NCCL_* / RCCL_* environment.  Times are the max over ranks."""
    import torch
    import torch.distributed as dist

    def timed(fn, iters):
        fn()
        sync()
        t = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        e = torch.tensor([(time.perf_counter() - t) / iters], dtype=torch.float64,
                         device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return float(e.item())

    world = dist.get_world_size()
    res = {}
    if engine == "native":
        eng = loop.ddp_model
        nbytes = eng.space.grad_flat.numel() * 4
        sec = timed(eng.reduce_all_now, 3)
        res["grad_reduce_all"] = {"mb": round(nbytes / 2**20, 1), "ms": round(sec * 1e3, 3),
                                  "busbw_GBps": round(nbytes / sec / 1e9 * 2 * (world - 1) / world, 1),
                                  "buckets": len(eng.buckets)}
        eng.zero_grad()
    sizes = (1, 4, 16, 32, 64, 128) if dev.type == "cuda" else (1, 4)
    res["pg_allreduce"] = []
    for mb in sizes:
        x = torch.ones(mb * (1 << 18), dtype=torch.float32, device=dev if dev.type == "cuda" else "cpu")
        sec = timed(lambda: dist.all_reduce(x), 5)
        res["pg_allreduce"].append({"mb": mb, "us": round(sec * 1e6, 1),
                                    "busbw_GBps": round(mb * 2**20 / sec / 1e9 * 2 * (world - 1) / world, 1)})
    # the RCCL knobs this run saw (none set = RCCL's own topology-derived defaults)
    res["rccl_env"] = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}
    return res


def project(a, loop, one_step, timed, exec_used, base):
    """One-GPU projection of W > 1: the same process's trainer with its
    DDP engine on the SIMULATED data plane (csrc/comm_sim.hip) - every bucket's all-reduce is a
    kernel on the reducer's high-priority comm stream that holds `cus` CUs for the link model's
    time and moves the ring's local HBM bytes.  The step math stays world 1.  Each (spec, wire,
    schedule) alternates a plain segment (no data plane) and a simulated one, --project-reps
    times, so clock drift over the run cancels: reported are the medians, the exposed comm
    (median of the paired differences), the exposed tail after the backward's last kernel, the
    grad-ready -> start delay (CU contention with the persistent GEMMs) and the link model's
    total comm time."""
    import statistics

    import torch
    eng = loop.ddp_model
    out = []
    wires = [w for w in a.project_wire.replace("/", ",").split(",") if w] or [a.grad_wire]
    scheds = [x for x in a.project_schedules.replace("/", ",").split(",") if x]

    def seg(sch, sim):
        if sch == "fused":
            loop.exec_microbatch, n = exec_used, a.steps
        else:
            loop.exec_microbatch, n = a.microbatch, a.ref_steps or 8
        for _ in range(2):  # untimed: a fresh reducer's / schedule's first steps
            one_step()
        if sim:
            eng.sim_stats(reset=True)
        h0 = dict(getattr(loop, "host_time", {}))
        e = timed(n) / n * 1e3
        host.append({k: round((v - h0.get(k, 0.0)) / n * 1e3, 2) for k, v in getattr(loop, "host_time", {}).items()})
        return e

    host = []  # per segment: the trainer's host ms per step (fwd / bwd enqueue), plain and sim alternating
    for spec in [x for x in a.project.split(";") if x.strip()]:
        f = [float(v) for v in spec.replace("/", ",").split(",")]
        world, bw = int(f[0]), f[1]
        cus = int(f[2]) if len(f) > 2 else 64
        lat = f[3] if len(f) > 3 else 10.0
        cap = f[4] if len(f) > 4 else None
        first = f[5] if len(f) > 5 else None
        for wire in wires:
            row = {"spec": None, "schedules": {}}
            for sch in scheds:
                plain, simt, stats = [], [], []
                host.clear()
                for _ in range(max(1, a.project_reps)):
                    eng.disable_sim_comm()
                    loop.use_ddp = False
                    plain.append(seg(sch, False))
                    eng.reduce_dtype = torch.bfloat16 if wire == "bf16" else torch.float32
                    info = eng.enable_sim_comm(world, bw, cus=cus, lat_us=lat, bucket_cap_mb=cap,
                                               first_bucket_mb=first)
                    row["spec"] = dict(info)
                    loop.use_ddp = True
                    simt.append(seg(sch, True))
                    stats.append(eng.sim_stats(reset=True))
                st = dict(stats[-1])
                for k in ("exposed_tail_ms", "ready_to_start_ms", "bucket_busy_ms", "comm_span_ms"):
                    st[k] = round(statistics.median(x[k] for x in stats), 3)
                st["last_step_timeline_ms"] = eng.sim_timeline()
                ms, pl = statistics.median(simt), statistics.median(plain)
                row["schedules"][sch] = dict(st, projected_ms_per_step=round(ms, 3), plain_ms_per_step=round(pl, 3),
                                             plain_runs=[round(x, 2) for x in plain],
                                             sim_runs=[round(x, 2) for x in simt],
                                             exposed_comm_ms=round(statistics.median(
                                                 s_ - p_ for s_, p_ in zip(simt, plain)), 3),
                                             projected_value=round(world / (ms / 1e3), 4),
                                             host_ms_per_step={"plain": host[0::2], "sim": host[1::2]})
                print(f"[bench] projection W={world} {bw} GB/s {wire} {sch}: {ms:.2f} ms/step "
                      f"(plain {pl:.2f}), tail {st['exposed_tail_ms']} ms", file=sys.stderr, flush=True)
                eng.disable_sim_comm()
                loop.use_ddp = False
            out.append(row)
    eng.reduce_dtype = torch.bfloat16 if a.grad_wire == "bf16" else torch.float32
    loop.exec_microbatch = exec_used
    return {"kind": "PROJECTION (one GPU, simulated data plane; not a scaling measurement)",
            "link_model": "busbw per spec; ring time = lat + 2 (W-1)/W x bucket bytes / busbw; the stand-in "
                          "kernel also reads and writes back 2 (W-1)/W x the bucket bytes",
            "base_ms_per_step": base, "reps": a.project_reps, "runs": out}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    from basic_utils import dist_util, logger
    from data import load_data_from_args
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop, LMTrainLoop

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        dist_util.setup_dist(silent=True)
    rank, world = dist_util.get_rank(), dist_util.get_world_size()
    if a.gpus != world and rank == 0:
        print(f"<WARN> --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = dist_util.dev()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        dist_util.claim_stream_plan(dev)  # world 1: before anything else takes a queue

    ref = a.reference_equivalent
    precision = a.precision or ("fp32" if ref else "bf16")
    engine = "torch" if ref else "native"
    exec_mb = a.exec_microbatch if a.exec_microbatch is not None else (-1 if ref else 0)

    logdir = tempfile.mkdtemp(prefix="dpa_bench_")
    logger.configure(dir=logdir, format_strs=["log"] if rank == 0 else [])
    seed_all(102)
    settings = dict(model=a.model, precision=precision, config_name=a.config_name,
                    seq_len=a.seq_len, vocab_size=30522 if a.model != "gpt2" else 50257,
                    hidden_dim=128, hidden_t_dim=128, dropout=0.1, use_hip_kernels=not a.stock)
    model = create_model_from_config(**settings).to(dev)
    n_params = sum(p.numel() for p in model.parameters())
    data = load_data_from_args("train", "synthetic", a.batch_size, deterministic=False, loop=True,
                               num_loader_proc=a.data_workers, dataset="synthetic",
                               seq_len=a.seq_len, vocab_size=settings["vocab_size"], seed=102 + rank,
                               model=a.model)
    kw = dict(model=model, data=data, batch_size=a.batch_size, microbatch=a.microbatch, lr=1e-4,
              ema_rate="0.5,0.9,0.99", log_interval=a.log_interval, save_interval=10 ** 9,
              resume_checkpoint="", weight_decay=0.0, learning_steps=320000,
              checkpoint_path=logdir, gradient_clipping=0.0, ddp_engine=engine,
              precision=precision, bucket_cap_mb=a.bucket_cap_mb,
              first_bucket_mb=a.first_bucket_mb, exec_microbatch=exec_mb,
              shard_optimizer=bool(a.zero1),
              grad_reduce_dtype=a.grad_wire)
    if a.model == "gpt2":
        loop = LMTrainLoop(**kw)
    else:
        diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000, noise_schedule="sqrt")
        loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, **kw)

    def one_step():
        batch = next(loop.data)
        loop.run_step(batch)
        if loop.step % loop.log_interval == 0:
            logger.dumpkvs()
        loop.step += 1

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist_util.barrier()

    t_w = time.time()
    for i in range(a.warmup):
        one_step()
        if rank == 0:  # progress (outside the timed region) for long or profiled runs
            print(f"[bench] warmup step {i + 1}/{a.warmup} queued at {time.time() - t_w:.1f} s",
                  file=sys.stderr, flush=True)
    sync()
    warm_s = time.time() - t_w
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_step()
    sync()
    elapsed = time.perf_counter() - t0
    rank_ms = [elapsed / a.steps * 1e3] * 2  # [min, max] over ranks of this rank's ms/step
    if world > 1:
        t = torch.tensor([elapsed, -elapsed], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        rank_ms = [-float(t[1].item()) / a.steps * 1e3, elapsed / a.steps * 1e3]

    exec_used = loop.exec_microbatch

    host = [0.0]  # host time to enqueue the last timed window (before its closing sync)

    def timed(n):
        sync()
        t = time.perf_counter()
        for _ in range(n):
            one_step()
        host[0] = time.perf_counter() - t
        sync()
        e = time.perf_counter() - t
        if world > 1:
            tt = torch.tensor([e], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            e = float(tt.item())
        return e

    ref_sched = None
    if a.ref_steps > 0 and not ref and exec_used != a.microbatch:
        # the reference's own schedule: one fwd/bwd per 64-sample micro-batch, no_sync on
        # all but the last (same model, optimizer state and process)
        loop._exec_auto = False
        loop.exec_microbatch = a.microbatch
        loop.cuda_graph = bool(a.ref_graph) and dev.type == "cuda"
        # (graph mode: two eager steps, then the capture + first replay - all untimed)
        for _ in range(max(3 if loop.cuda_graph else 1, a.ref_warmup)):
            one_step()
        diag = []
        if a.ref_windows > 1:  # per-window diagnostics: allocator growth and Python GC time
            import gc
            gc_t = [0.0, 0.0]

            def _gc_cb(phase, info):
                if phase == "start":
                    gc_t[1] = time.perf_counter()
                else:
                    gc_t[0] += time.perf_counter() - gc_t[1]
            gc.callbacks.append(_gc_cb)

        def win():
            if a.ref_windows <= 1 or dev.type != "cuda":
                return timed(a.ref_steps)
            m0 = torch.cuda.memory_stats(dev)
            g0 = gc_t[0]
            h0 = dict(getattr(loop, "host_time", {}))
            e = timed(a.ref_steps)
            m1 = torch.cuda.memory_stats(dev)
            diag.append({k: m1.get(k, 0) - m0.get(k, 0) for k in ("num_device_alloc", "num_device_free",
                                                                  "num_alloc_retries")})
            diag[-1]["gc_ms"] = round((gc_t[0] - g0) * 1e3, 1)
            diag[-1]["host_ms_per_step"] = round(host[0] / a.ref_steps * 1e3, 1)
            for k, v in getattr(loop, "host_time", {}).items():
                diag[-1][f"host_{k}_ms_per_step"] = round((v - h0.get(k, 0.0)) / a.ref_steps * 1e3, 1)
            diag[-1]["alloc_gb"] = round(torch.cuda.memory_allocated(dev) / 2 ** 30, 2)
            diag[-1]["reserved_gb"] = round(torch.cuda.memory_reserved(dev) / 2 ** 30, 2)
            return e
        wins = [win() for _ in range(max(1, a.ref_windows))]
        e, n_ref = sum(wins), a.ref_steps * len(wins)
        ref_sched = {"exec_microbatch": a.microbatch, "steps": n_ref,
                     "hip_graph": loop._graph is not None,
                     "ms_per_step": round(e / n_ref * 1e3, 3),
                     "value": round(n_ref / e * world, 4)}
        if len(wins) > 1:
            ref_sched["windows_ms"] = [round(w / a.ref_steps * 1e3, 2) for w in wins]
            ref_sched["windows_diag"] = diag

    projection = None
    if a.project and world == 1 and engine == "native" and dev.type == "cuda":
        base = {"fused": round(elapsed / a.steps * 1e3, 3),
                "reference": ref_sched["ms_per_step"] if ref_sched else None}
        projection = project(a, loop, one_step, timed, exec_used, base)
        loop._exec_auto = False

    ms = elapsed / a.steps * 1e3
    steps_per_s = a.steps / elapsed
    value = steps_per_s * world
    samples_per_s = steps_per_s * a.batch_size * world
    baseline = stock = None
    bpath = os.path.join(HERE, "baseline_measured.json")
    headline = (a.model == "diffuseq" and a.config_name == "bert-base-uncased" and a.seq_len == 128
                and a.batch_size == 2048 and a.microbatch == 64)
    if os.path.exists(bpath) and not ref and not a.stock and headline:
        with open(bpath) as f:
            b = json.load(f)
        per_gpu = b.get("reference_equivalent_steps_per_sec_per_gpu")
        if per_gpu:
            baseline = per_gpu * world
        # the best stock-PyTorch bf16 run of the reference's trainer (micro-batch 64 or fused)
        sb = b.get("stock_bf16_steps_per_sec_per_gpu")
        if sb:
            stock = sb * world
    out = {
        # the BASELINE.json metric for the headline config; other configs say what they ran
        "metric": METRIC if headline else (f"train steps/sec (whole node), {a.model}/{a.config_name} "
                                            f"seq{a.seq_len} bs{a.batch_size} DDP on MI355X"),
        "value": round(value, 4),
        "unit": f"steps/s summed over GPUs (1 step = {a.batch_size} samples x {a.seq_len} tokens per GPU)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / baseline, 3) if baseline else None,
        "vs_stock_bf16": round(value / stock, 3) if stock else None,
        "dtype": "bf16" if precision == "bf16" else "fp32",
        "data": "synthetic (random token ids, random src/trg split; random-init weights)",
        "config": {"model": "DiffuSeq-base" if a.config_name == "bert-base-uncased" else a.config_name,
                   "global_batch": a.batch_size * world, "per_gpu_batch": a.batch_size,
                   "microbatch": a.microbatch, "exec_microbatch": exec_used,
                   "seq_len": a.seq_len, "parallelism": f"dp{world}",
                   "engine": engine, "params": n_params, "stock_ops": bool(a.stock)},
        "optimizer_steps_per_sec": round(steps_per_s, 4),
        "samples_per_sec": round(samples_per_s, 1),
        "tokens_per_sec": round(samples_per_s * a.seq_len, 1),
        "warmup_s": round(warm_s, 2),
        "schedule": ("fused: %d micro-batches of %d per executed fwd/bwd (gradient = reference sum)"
                     % (exec_used // a.microbatch, a.microbatch)) if exec_used != a.microbatch
                    else "reference: one fwd/bwd per micro-batch",
        "reference_schedule": ref_sched,
    }
    if projection is not None:
        out["projection"] = projection
    if engine == "native":
        out["config"]["bucket_mb"] = loop.ddp_model.bucket_sizes_mb()
        if loop.ddp_model.bucket_tune is not None:
            out["config"]["bucket_tune"] = dict({"cap_mb": loop.ddp_model.bucket_cap_mb,
                                                 "first_mb": loop.ddp_model.first_bucket_mb},
                                                **loop.ddp_model.bucket_tune)
        nat = getattr(loop.ddp_model, "_native", None)
        direct = nat is not None and nat.direct()
        out["config"]["comm"] = ("reducer-owned RCCL communicator on the stream plan's comm stream (pooled "
                                 "queue, priority %d)" % nat.stream_priority()
                                 if direct else ("c10d process group" if world > 1 else "none (world 1)"))
        # where each collective of a W > 1 step runs (the W > 1 resource plan)
        eng_ = loop.ddp_model
        out["config"]["data_plane"] = {
            "bucket_reduce": out["config"]["comm"],
            "bucket_tuning": ((eng_.bucket_tune or {}).get("timed_on") or
                              ("fixed sizes (--bucket-cap-mb)" if a.bucket_cap_mb > 0 else "none (world 1)")),
            "zero1_param_gather": ("n/a" if not eng_.sharded else
                                   "reducer-owned RCCL communicator, comm stream" if direct else "process group"),
            "control_plane": "process group (loss / grad-norm logging means, checksums)" if world > 1 else "none"}
    # evidence of what the job ran on: the backend's world size, the ranks of the communicator
    # the gradient buckets are reduced over (the reducer-owned RCCL communicator's
    # ncclCommCount in direct mode), and the spread of per-rank step times
    out["ranks"] = {"backend": dist.get_backend() if world > 1 else None,
                    "backend_world_size": dist.get_world_size() if world > 1 else 1,
                    "data_plane_comm_ranks": (loop.ddp_model.comm_ranks()
                                              if engine == "native" else world),
                    "rank_ms_per_step_min": round(rank_ms[0], 3),
                    "rank_ms_per_step_max": round(rank_ms[1], 3)}
    if world > 1 and a.comm_probe:
        try:  # diagnostics only: never cost the measured line
            out["comm_probe"] = comm_probe(loop, engine, dev, sync)
        except Exception as e:  # noqa: BLE001
            out["comm_probe"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if dev.type == "cuda":  # HBM headroom of the fused schedule (288 GB per MI355X)
        out["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
        free, total = torch.cuda.mem_get_info(dev)
        out["hbm_free_gb"] = round(free / 2**30, 1)  # device-wide free now (RCCL buffers excluded)
        out["hbm_total_gb"] = round(total / 2**30, 1)
        # headroom at the step's peak: what the caching allocator never had to reserve (RCCL's
        # lazily allocated buffers live there), and how often it freed its cache and retried
        # a failed hipMalloc (steps thrashing at the edge of HBM)
        ms = torch.cuda.memory_stats(dev)
        out["hbm_headroom_at_peak_gb"] = round((total - torch.cuda.max_memory_reserved(dev)) / 2**30, 1)
        out["alloc_retries"] = int(ms.get("num_alloc_retries", 0))
    if dev.type == "cuda":  # the step's stream plan (runtime/streams.py): role -> stream id
        from distributed_pipeline_amd.runtime.streams import StreamPlan
        out["streams"] = StreamPlan.for_device(dev).describe()
        nat = getattr(getattr(loop, "ddp_model", None), "_native", None)
        if nat is not None and hasattr(nat, "comm_stream") and nat.direct():
            out["streams"]["handles"]["comm"] = hex(nat.comm_stream())
    if rank == 0:
        out["topology"] = topology()
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
