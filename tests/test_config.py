"""Settings DSL: argparse/JSON round trips (reference config/base.py, config/train.py)."""
import json
import subprocess
import sys

import pytest

from config.base import C, S, _, bool_validator
from config.train import TrainSettings

REF_ORDER = ["lr", "batch_size", "microbatch", "learning_steps", "log_interval", "save_interval",
             "eval_interval", "ema_rate", "seed", "resume_checkpoint", "checkpoint_path",
             "gradient_clipping", "weight_decay", "dataset", "data_dir", "data_loader_workers"]


def test_reference_fields_defaults_and_order():
    d = TrainSettings().dict()
    assert list(d)[:len(REF_ORDER)] == REF_ORDER
    assert d["lr"] == 1e-4 and d["batch_size"] == 2048 and d["microbatch"] == 64
    assert d["learning_steps"] == 320000 and d["ema_rate"] == "0.5,0.9,0.99" and d["seed"] == 102


def test_json_round_trip_and_override(tmp_path):
    cfg = tmp_path / "c.json"
    cfg.write_text(TrainSettings(lr=3e-4, batch_size=32).json(indent=2))
    p = TrainSettings.to_argparse(add_json=True)
    ns = p.parse_args(["--config_json", str(cfg)])
    s = TrainSettings.from_argparse(ns)
    assert s.lr == 3e-4 and s.batch_size == 32
    # explicit flags override the JSON (reference silently ignored them, C6)
    ns = p.parse_args(["--config_json", str(cfg), "--batch_size", "16", "--seed", "7"])
    s = TrainSettings.from_argparse(ns)
    assert s.batch_size == 16 and s.seed == 7 and s.lr == 3e-4


def test_multiple_cli_flags_allowed():
    p = TrainSettings.to_argparse(add_json=True)
    s = TrainSettings.from_argparse(p.parse_args(["--lr", "0.001", "--batch_size", "8",
                                                  "--predict_xstart", "no", "--model", "gpt2"]))
    assert s.lr == 1e-3 and s.batch_size == 8 and s.predict_xstart is False and s.model == "gpt2"


def test_extra_json_keys_rejected(tmp_path):
    cfg = tmp_path / "c.json"
    d = TrainSettings().dict()
    d["not_a_field"] = 1
    cfg.write_text(json.dumps(d))
    p = TrainSettings.to_argparse(add_json=True)
    with pytest.raises(Exception):
        TrainSettings.from_argparse(p.parse_args(["--config_json", str(cfg)]))


def test_bad_choice_rejected():
    p = TrainSettings.to_argparse(add_json=True)
    with pytest.raises(SystemExit):
        p.parse_args(["--model", "resnet"])


@pytest.mark.parametrize("text,val", [("yes", True), ("true", True), ("1", True), ("off", False),
                                      ("no", False), ("0", False)])
def test_bool_validator(text, val):
    assert bool_validator(text) is val


def test_nested_groups_work():
    """The reference's __main__ demo (config/base.py:90-107) crashed on nested groups (C5)."""
    class Config1(S):
        a: int = _(1, description="this is a")
        b: int = _(2, description="this is b")

    class Config2(S):
        c: C("choice1", "choice2") = _("choice2", description="this is c")
        d: bool = _(True, description="this is d")

    class Config(S):
        conf1: Config1 = Config1()
        conf2: Config2 = Config2()

    cfg = Config.from_argv(["--a", "5", "--c", "choice1", "--d", "false"])
    assert cfg.conf1.a == 5 and cfg.conf1.b == 2 and cfg.conf2.c == "choice1" and cfg.conf2.d is False


def test_readme_copy_config_one_liner():
    out = subprocess.run([sys.executable, "-c",
                          "from config.train import TrainSettings as T; print(T().json(indent=2))"],
                         capture_output=True, text=True, check=True).stdout
    assert json.loads(out)["batch_size"] == 2048
