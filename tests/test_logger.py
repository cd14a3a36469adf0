"""KV logger formats and semantics (reference basic_utils/logger.py; SURVEY O-1..O-10, Q6, Q7)."""
import json
import os

import torch

from basic_utils import logger


def test_human_format_golden(tmp_path):
    logger.configure(dir=str(tmp_path), format_strs=["log"])
    logger.logkv("step", 3)
    logger.logkv("a_long_key_name", 0.123456)
    logger.logkv("B", "text")
    logger.dumpkvs()
    text = (tmp_path / "log.txt").read_text().splitlines()
    assert text[0] == "Logging to %s" % tmp_path
    table = text[1:]
    assert table[0] == "-" * len(table[1]) and table[-1] == table[0]
    assert table[1:-1] == ["| a_long_key_name | 0.123    |",
                           "| B               | text     |",
                           "| step            | 3        |"]


def test_csv_header_grows(tmp_path):
    logger.configure(dir=str(tmp_path), format_strs=["csv"])
    logger.logkv("a", 1)
    logger.dumpkvs()
    logger.logkv("a", 2)
    logger.logkv("b", 3)
    logger.dumpkvs()
    lines = (tmp_path / "progress.csv").read_text().splitlines()
    assert lines == ["a,b", "1,", "2,3"]


def test_json_and_mean_with_device_tensors(tmp_path):
    logger.configure(dir=str(tmp_path), format_strs=["json"])
    logger.logkv_mean("loss", torch.tensor(1.0))
    logger.logkv_mean("loss", torch.tensor(3.0))
    logger.logkv_mean("x", 1.0)
    logger.logkv_mean("x", 2.0)
    out = logger.dumpkvs()
    assert out["loss"] == 2.0 and out["x"] == 1.5
    row = json.loads((tmp_path / "progress.json").read_text().splitlines()[0])
    assert row == {"loss": 2.0, "x": 1.5}


def test_profile_kv_accumulates(tmp_path):
    logger.configure(dir=str(tmp_path), format_strs=[])
    with logger.profile_kv("io"):
        pass
    assert "wait_io" in logger.getkvs()


def test_append_mode_keeps_history(tmp_path):
    logger.configure(dir=str(tmp_path), format_strs=["log", "csv"])
    logger.logkv("k", 1)
    logger.dumpkvs()
    logger.configure(dir=str(tmp_path), format_strs=["log", "csv"], append=True)
    logger.logkv("k", 2)
    logger.dumpkvs()
    csv = (tmp_path / "progress.csv").read_text().splitlines()
    assert csv == ["k", "1", "2"]
    assert (tmp_path / "log.txt").read_text().count("| k ") == 2


def test_rank_suffix_from_RANK(tmp_path, monkeypatch):
    monkeypatch.setenv("RANK", "3")
    logger.configure(dir=str(tmp_path))
    assert os.path.exists(tmp_path / "log-rank003.txt")
    monkeypatch.delenv("RANK")
    logger.configure(dir=str(tmp_path), format_strs=[])


def test_tensorboard_events_roundtrip(tmp_path):
    """Built-in event writer: valid TFRecord framing (CRC32C) + decodable scalars."""
    from basic_utils import tb_events
    assert tb_events.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    fmt = logger.make_output_format("tensorboard", str(tmp_path))
    fmt.writekvs({"loss": 1.5, "step": 3, "name": "x"})
    fmt.writekvs({"loss": 0.25})
    fmt.close()
    files = list((tmp_path / "tb").glob("events.out.tfevents.*"))
    assert len(files) == 1
    ev = tb_events.read_events(str(files[0]))
    assert ev[0][0] == 1 and abs(ev[0][1]["loss"] - 1.5) < 1e-6 and ev[0][1]["step"] == 3.0
    assert ev[1] == (2, {"loss": 0.25})
