"""End-to-end launcher tests on CPU/gloo (BASELINE config #1): the reference entry point
``python -m run.train --distributed --config_json ...`` with world_size 2, and an
elastic restart after an injected rank crash resuming from the checkpoint dir
(SURVEY CS-1, 5.3, 5.4)."""
import os
import subprocess
import sys

import torch

from basic_utils.dist_util import find_free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, extra_env=None, extra_args=()):
    env = dict(os.environ)
    env.pop("LOCAL_RANK", None)
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT, **(extra_env or {}))
    cmd = [sys.executable, "-m", "run.train", "--distributed", "--nproc_per_node", "2",
           "--master_addr", "127.0.0.1", "--master_port", str(find_free_port()),
           "--config_json", os.path.join(ROOT, "configs", "tiny_mlp_cpu.json"),
           "--checkpoint_path", str(tmp_path / "ck"), "--learning_steps", "4",
           "--save_interval", "1", "--log_interval", "1", *extra_args]
    return subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                          timeout=240)


def test_two_rank_cpu_run_writes_reference_layout(tmp_path):
    r = _run(tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    names = set(os.listdir(tmp_path / "ck"))
    for n in range(1, 4):
        assert {f"model_{n:06d}.pt", f"opt_{n:06d}.pt", f"ema_0.9_{n:06d}.pt"} <= names
    assert "training_args.json" in names and "progress.csv" in names
    sd = torch.load(tmp_path / "ck" / "model_000003.pt", weights_only=True)
    assert all(torch.isfinite(v).all() for v in sd.values())


def test_elastic_restart_after_injected_crash_resumes(tmp_path):
    r = _run(tmp_path, extra_env={"DP_FAULT_AT_STEP": "2", "DP_FAULT_RANK": "1"},
             extra_args=("--max_restarts", "1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "exitcode: 17" in out                          # the injected crash happened
    assert "loading model from checkpoint" in out and "model_000001.pt" in out  # resumed
    assert (tmp_path / "ck" / ".fault_injected_2").exists()
    assert (tmp_path / "ck" / "model_000003.pt").exists()  # and finished


def test_allreduce_sweep_tool_runs_on_gloo_ranks():
    """tools/bench_allreduce.py (bucket-size sweep) on 2 CPU ranks."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(find_free_port()),
                          os.path.join(root, "tools", "bench_allreduce.py"), "--backend", "gloo",
                          "--sizes-mb", "0.25,1", "--iters", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert [r["size_mb"] for r in rows] == [0.25, 1.0]
    assert all(r["world"] == 2 and r["algbw_GBps"] > 0 for r in rows)


def test_bench_contract_two_ranks_gloo():
    """bench.py under torch.distributed.run exactly as the round driver launches it
    (tiny config on CPU ranks): rank 0 prints ONE JSON line with the whole-job value."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(find_free_port()),
                          os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--config-name", "tiny", "--batch-size", "8", "--microbatch", "4", "--seq-len", "64",
                          "--data-workers", "0"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 16
    assert abs(d["value"] - 2 * d["optimizer_steps_per_sec"]) < 1e-3 * d["value"]
    assert abs(d["ms_per_step"] - 1e3 / d["optimizer_steps_per_sec"]) < 1e-2 * d["ms_per_step"]
    # the BASELINE metric / ratio belong to the headline config only
    assert d["vs_baseline"] is None and "tiny" in d["metric"]
    # rank evidence and the post-run comm probe (N > 1)
    assert d["ranks"]["backend_world_size"] == 2 and d["ranks"]["data_plane_comm_ranks"] == 2
    cp = d["comm_probe"]
    assert cp["grad_reduce_all"]["ms"] > 0 and cp["grad_reduce_all"]["buckets"] >= 1
    assert [r["mb"] for r in cp["pg_allreduce"]] == [1, 4] and all(r["busbw_GBps"] > 0 for r in cp["pg_allreduce"])
    # bucket sizes measured at startup (bench default bucket_cap_mb=0): the cap is a swept size
    bt = d["config"]["bucket_tune"]
    assert bt["cap_mb"] in [r["mb"] for r in bt["sweep"]] and bt["first_mb"] <= bt["cap_mb"]
    assert all(r["busbw_GBps"] > 0 for r in bt["sweep"])
