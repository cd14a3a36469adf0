"""The real entry point on the GPU (SURVEY CS-1, reference train.sh:1 / run/train.py:124-126):
``python -m run.train --distributed --nproc_per_node 1 --config_json <tiny DiffuSeq, bf16>``
through dist_run -> torchrun -> one worker on RCCL, native engine and kernels; then a
second launch auto-resumes from the checkpoint directory and finishes the schedule."""
import os
import subprocess
import sys

import pytest
import torch

from basic_utils.dist_util import find_free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _launch(tmp_path, steps):
    env = dict(os.environ)
    env.pop("LOCAL_RANK", None)
    env.update(PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", WANDB_MODE="disabled")
    cmd = [sys.executable, "-u", "-m", "run.train", "--distributed", "--nproc_per_node", "1",
           "--master_addr", "127.0.0.1", "--master_port", str(find_free_port()),
           "--config_json", os.path.join(ROOT, "configs", "tiny_diffuseq_gpu.json"),
           "--checkpoint_path", str(tmp_path / "ck"), "--learning_steps", str(steps)]
    return subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=100)


def test_run_train_rccl_world1_saves_and_resumes(tmp_path):
    r = _launch(tmp_path, 4)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "torch.distributed setup success" in out
    names = set(os.listdir(tmp_path / "ck"))
    assert "model_000002.pt" in names and "opt_000002.pt" in names, names
    last = max(int(n[6:12]) for n in names if n.startswith("model_"))
    sd = torch.load(tmp_path / "ck" / f"model_{last:06d}.pt", weights_only=True)
    assert all(torch.isfinite(v).all() for v in sd.values())
    r2 = _launch(tmp_path, 7)
    out2 = r2.stdout + r2.stderr
    assert r2.returncode == 0, out2[-4000:]
    assert "loading model from checkpoint" in out2 and f"model_{last:06d}.pt" in out2
    names2 = set(os.listdir(tmp_path / "ck"))
    assert max(int(n[6:12]) for n in names2 if n.startswith("model_")) > last
    with open(tmp_path / "ck" / "progress.csv") as f:
        rows = f.read().strip().splitlines()
    assert len(rows) >= 4 and "loss" in rows[0]
