"""
Key/value + text logger (L3), API-compatible with the reference
``basic_utils/logger.py`` (reference: basic_utils/logger.py:18-500, itself the
OpenAI-baselines logger).  Same free-function API (``logkv``, ``logkv_mean``,
``dumpkvs``, ``log``, ``configure``, ``profile_kv`` ...) and the same
stdout/log/csv/json output formats byte-for-byte.

What is different, and why:

* **Device-lazy values.**  ``logkv``/``logkv_mean`` accept torch tensors (e.g. a
  loss living on the GPU) and keep them on the device; the running mean is an
  on-device (sum, count) pair and the single device->host copy happens in
  ``dumpkvs``, i.e. once per ``log_interval`` instead of once per micro-batch
  (reference trainer.py:265-271 did one ``.item()`` per parameter per step).
* **Ranks.**  The writer rank is the *global* rank (``RANK``), not the MPI env
  vars only (every torchrun rank used to write the same log.txt).
* **Cross-rank mean.**  ``configure(comm="dist")`` (or ``set_comm("dist")``)
  averages every key over ranks with ONE packed all-reduce at dump time
  (replaces the dead ``mpi_weighted_mean`` path, SURVEY X-6).
* **Resume.**  ``configure(..., append=True)`` appends to existing files
  instead of truncating them.
* **TensorBoard** goes through ``torch.utils.tensorboard`` when available
  (the TF1 writer of the reference is dead code on TF2).
* ``wandb`` is optional and only the global rank 0 logs to it.
"""

from abc import ABC, abstractmethod
import datetime
import json
import os
import sys
import tempfile
import time
from collections import defaultdict
from contextlib import contextmanager

DEBUG = 10
INFO = 20
WARN = 30
ERROR = 40
DISABLED = 50


# ============================================================================
# Output formats
# ============================================================================

class KVWriter(ABC):
    @abstractmethod
    def writekvs(self, kvs):
        raise NotImplementedError


class SeqWriter(ABC):
    @abstractmethod
    def writeseq(self, seq):
        raise NotImplementedError


def _fmt_value(val):
    if hasattr(val, "__float__"):
        return "%-8.3g" % val
    return str(val)


def _clip30(text):
    return text if len(text) <= 30 else text[:27] + "..."


class HumanOutputFormat(KVWriter, SeqWriter):
    """Aligned ``| key | value |`` table (stdout and ``log.txt``)."""

    def __init__(self, filename_or_file, mode="wt"):
        if isinstance(filename_or_file, str):
            self.file = open(filename_or_file, mode)
            self.own_file = True
        else:
            assert hasattr(filename_or_file, "write"), \
                "expected file or str, got %s" % filename_or_file
            self.file = filename_or_file
            self.own_file = False

    def writekvs(self, kvs):
        cells = {_clip30(k): _clip30(_fmt_value(v)) for k, v in sorted(kvs.items())}
        if not cells:
            print("WARNING: tried to write empty key-value dict")
            return
        kw = max(len(k) for k in cells)
        vw = max(len(v) for v in cells.values())
        bar = "-" * (kw + vw + 7)
        rows = [bar]
        for k in sorted(cells, key=str.lower):
            rows.append("| " + k.ljust(kw) + " | " + cells[k].ljust(vw) + " |")
        rows.append(bar)
        self.file.write("\n".join(rows) + "\n")
        self.file.flush()

    @staticmethod
    def _truncate(s):
        return _clip30(s)

    def writeseq(self, seq):
        self.file.write(" ".join(list(seq)) + "\n")
        self.file.flush()

    def close(self):
        if self.own_file:
            self.file.close()


class JSONOutputFormat(KVWriter):
    """One JSON object per dump (``progress.json``)."""

    def __init__(self, filename, mode="wt"):
        self.file = open(filename, mode)

    def writekvs(self, kvs):
        row = {k: (float(v) if hasattr(v, "dtype") else v) for k, v in sorted(kvs.items())}
        self.file.write(json.dumps(row) + "\n")
        self.file.flush()

    def close(self):
        self.file.close()


class CSVOutputFormat(KVWriter):
    """``progress.csv``; the header grows (and the file is rewritten) when new keys appear."""

    def __init__(self, filename, mode="w+t"):
        existed = os.path.exists(filename) and mode.startswith("a")
        self.file = open(filename, "r+t" if existed else "w+t")
        self.keys = []
        self.sep = ","
        if existed:
            header = self.file.readline().rstrip("\n")
            self.keys = header.split(self.sep) if header else []
            self.file.seek(0, os.SEEK_END)

    def _rewrite_with_new_keys(self, new_keys):
        self.file.seek(0)
        old_rows = self.file.readlines()[1:]
        self.keys.extend(new_keys)
        self.file.seek(0)
        self.file.truncate()
        self.file.write(self.sep.join(self.keys) + "\n")
        pad = self.sep * len(new_keys)
        for line in old_rows:
            self.file.write(line.rstrip("\n") + pad + "\n")

    def writekvs(self, kvs):
        new_keys = sorted(set(kvs) - set(self.keys))
        if new_keys:
            self._rewrite_with_new_keys(new_keys)
        vals = []
        for k in self.keys:
            v = kvs.get(k)
            vals.append("" if v is None else str(v))
        self.file.write(self.sep.join(vals) + "\n")
        self.file.flush()

    def close(self):
        self.file.close()


class TensorBoardOutputFormat(KVWriter):
    """Scalars to TensorBoard: ``torch.utils.tensorboard`` when the ``tensorboard``
    package is installed, else the built-in event-file writer (``tb_events``)."""

    def __init__(self, dir):
        os.makedirs(dir, exist_ok=True)
        self.dir = dir
        self.step = 1
        self.writer = self.events = None
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.writer = SummaryWriter(log_dir=dir)
        except Exception:  # tensorboard not installed
            from .tb_events import EventFileWriter
            self.events = EventFileWriter(dir)

    def writekvs(self, kvs):
        scalars = {}
        for k, v in kvs.items():
            try:
                scalars[k] = float(v)
            except (TypeError, ValueError):
                pass
        if self.writer is not None:
            for k, v in scalars.items():
                self.writer.add_scalar(k, v, self.step)
            self.writer.flush()
        else:
            self.events.add_scalars(scalars, self.step)
        self.step += 1

    def close(self):
        if self.writer is not None:
            self.writer.close()
            self.writer = None
        if self.events is not None:
            self.events.close()
            self.events = None


def make_output_format(format, ev_dir, log_suffix="", append=False):
    os.makedirs(ev_dir, exist_ok=True)
    text_mode = "at" if append else "wt"
    if format == "stdout":
        return HumanOutputFormat(sys.stdout)
    if format == "log":
        return HumanOutputFormat(os.path.join(ev_dir, "log%s.txt" % log_suffix), text_mode)
    if format == "json":
        return JSONOutputFormat(os.path.join(ev_dir, "progress%s.json" % log_suffix), text_mode)
    if format == "csv":
        return CSVOutputFormat(os.path.join(ev_dir, "progress%s.csv" % log_suffix),
                               "a+t" if append else "w+t")
    if format == "tensorboard":
        return TensorBoardOutputFormat(os.path.join(ev_dir, "tb%s" % log_suffix))
    raise ValueError("Unknown format specified: %s" % (format,))


# ============================================================================
# Free-function API
# ============================================================================

def logkv(key, val):
    """Record ``val`` for ``key`` this iteration (last value wins)."""
    get_current().logkv(key, val)


def logkv_mean(key, val):
    """Record ``val`` for ``key``; repeated calls are averaged."""
    get_current().logkv_mean(key, val)


def logkv_mean_sum(key, total, count):
    """Record ``count`` values summing to ``total`` for ``key`` (as that many logkv_mean calls)."""
    get_current().logkv_mean_sum(key, total, count)


def logkvs(d):
    for k, v in d.items():
        logkv(k, v)


def dumpkvs():
    """Emit all recorded diagnostics and clear them."""
    return get_current().dumpkvs()


def getkvs():
    return get_current().name2val


def log(*args, level=INFO):
    get_current().log(*args, level=level)


def debug(*args):
    log(*args, level=DEBUG)


def info(*args):
    log(*args, level=INFO)


def warn(*args):
    log(*args, level=WARN)


def error(*args):
    log(*args, level=ERROR)


def set_level(level):
    get_current().set_level(level)


def set_comm(comm):
    get_current().set_comm(comm)


def get_dir():
    return get_current().get_dir()


record_tabular = logkv
dump_tabular = dumpkvs


@contextmanager
def profile_kv(scopename):
    """Add the wall time of the ``with`` body to key ``wait_<scopename>``."""
    key = "wait_" + scopename
    t0 = time.time()
    try:
        yield
    finally:
        get_current().name2val[key] += time.time() - t0


def profile(n):
    """Decorator form of :func:`profile_kv`."""
    def wrap(func):
        def inner(*args, **kwargs):
            with profile_kv(n):
                return func(*args, **kwargs)
        return inner
    return wrap


# ============================================================================
# Backend
# ============================================================================

# Callables ``hook(logger)`` run at the start of every ``Logger.dumpkvs`` (of any
# logger, including one configured later), so code that accumulates metrics on
# the device can publish them at log cadence without patching a logger instance.
_DUMP_HOOKS = []


def add_dump_hook(fn):
    """Register ``fn(logger)`` to run before each dump; idempotent per function."""
    if fn not in _DUMP_HOOKS:
        _DUMP_HOOKS.append(fn)
    return fn


def get_current():
    if Logger.CURRENT is None:
        _configure_default_logger()
    return Logger.CURRENT


def _is_tensor(x):
    return type(x).__module__.startswith("torch") and hasattr(x, "detach")


class _MeanAcc:
    """Running mean kept as (sum, count); sum may be a device tensor."""
    __slots__ = ("total", "count")

    def __init__(self):
        self.total = 0.0
        self.count = 0

    def add(self, val):
        if _is_tensor(val):
            val = val.detach().float()
            if val.dim() > 0:
                val = val.mean()
            self.total = val.clone() if not _is_tensor(self.total) and self.total == 0.0 \
                else self.total + val
        else:
            self.total = self.total + val
        self.count += 1

    def add_sum(self, total, count):
        """``count`` recorded values at once, given their sum (a device scalar or float)."""
        if _is_tensor(total):
            total = total.detach().float()
            self.total = total.clone() if not _is_tensor(self.total) and self.total == 0.0 \
                else self.total + total
        else:
            self.total = self.total + total
        self.count += count

    def value(self):
        return self.total / max(self.count, 1)


def _to_host(d):
    """Convert device tensors in ``d`` to python floats with one sync."""
    tensor_keys = [k for k, v in d.items() if _is_tensor(v)]
    if tensor_keys:
        import torch
        packed = torch.stack([d[k].detach().float().reshape(()) for k in tensor_keys]).cpu()
        for k, v in zip(tensor_keys, packed.tolist()):
            d[k] = v
    return d


def _global_rank():
    for var in ("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK"):
        if var in os.environ:
            return int(os.environ[var])
    return 0


class Logger(object):
    DEFAULT = None
    CURRENT = None

    def __init__(self, dir, output_formats, comm=None):
        self.name2val = defaultdict(float)   # last values (and profile_kv sums)
        self.name2cnt = defaultdict(int)
        self._means = {}                     # key -> _MeanAcc
        self.level = INFO
        self.dir = dir
        self.output_formats = output_formats
        self.comm = comm

    # -- logging API --------------------------------------------------------
    def logkv(self, key, val):
        self._means.pop(key, None)
        self.name2val[key] = val

    def logkv_mean_sum(self, key, total, count):
        """As ``count`` logkv_mean calls whose values sum to ``total``."""
        acc = self._means.get(key)
        if acc is None:
            acc = self._means[key] = _MeanAcc()
            if key in self.name2val and self.name2cnt.get(key, 0):
                acc.total = self.name2val[key] * self.name2cnt[key]
                acc.count = self.name2cnt[key]
        acc.add_sum(total, count)
        self.name2cnt[key] = acc.count
        if not _is_tensor(acc.total):
            self.name2val[key] = acc.value()

    def logkv_mean(self, key, val):
        acc = self._means.get(key)
        if acc is None:
            acc = self._means[key] = _MeanAcc()
            if key in self.name2val and self.name2cnt.get(key, 0):
                acc.total = self.name2val[key] * self.name2cnt[key]
                acc.count = self.name2cnt[key]
        acc.add(val)
        self.name2cnt[key] = acc.count
        if not _is_tensor(acc.total):  # device means are resolved lazily at dump
            self.name2val[key] = acc.value()

    def _collect(self):
        d = dict(self.name2val)
        for k, acc in self._means.items():
            d[k] = acc.value()
        return _to_host(d)

    def _cross_rank_mean(self, d):
        if self.comm is None:
            return d
        if self.comm == "dist":
            try:
                import torch
                import torch.distributed as dist
            except ImportError:
                return d
            if not (dist.is_available() and dist.is_initialized()):
                return d
            keys = sorted(k for k, v in d.items() if isinstance(v, (int, float)))
            device = torch.device("cpu")
            if dist.get_backend() == "nccl":
                device = torch.device("cuda", torch.cuda.current_device())
            buf = torch.zeros(2 * len(keys) + 1, dtype=torch.float64, device=device)
            for i, k in enumerate(keys):
                c = float(self.name2cnt.get(k, 1) or 1)
                buf[2 * i] = float(d[k]) * c
                buf[2 * i + 1] = c
            dist.all_reduce(buf)
            out = dict(d)
            vals = buf.cpu().tolist()
            for i, k in enumerate(keys):
                out[k] = vals[2 * i] / max(vals[2 * i + 1], 1e-12)
            return out
        # mpi4py-style communicator (reference semantics)
        return mpi_weighted_mean(self.comm, {k: (v, self.name2cnt.get(k, 1)) for k, v in d.items()})

    def dumpkvs(self):
        for hook in list(_DUMP_HOOKS):  # late-bound keys (e.g. device-side accumulators)
            hook(self)
        d = self._cross_rank_mean(self._collect())
        out = d.copy()
        if _global_rank() == 0:
            _wandb_log(d)
        if _global_rank() == 0:
            for fmt in self.output_formats:
                if isinstance(fmt, KVWriter) and d:
                    fmt.writekvs(d)
        self.name2val.clear()
        self.name2cnt.clear()
        self._means.clear()
        return out

    def log(self, *args, level=INFO):
        if self.level <= level:
            self._do_log(args)

    # -- configuration ------------------------------------------------------
    def set_level(self, level):
        self.level = level

    def set_comm(self, comm):
        self.comm = comm

    def get_dir(self):
        return self.dir

    def close(self):
        for fmt in self.output_formats:
            fmt.close()

    def _do_log(self, args):
        for fmt in self.output_formats:
            if isinstance(fmt, SeqWriter):
                fmt.writeseq(map(str, args))


def _wandb_log(d):
    try:
        import wandb  # optional
    except ImportError:
        return
    if getattr(wandb, "run", None) is not None:
        wandb.log(dict(d))


def get_rank_without_mpi_import():
    return _global_rank()


def mpi_weighted_mean(comm, local_name2valcount):
    """Weighted mean of {name: (value, count)} over an mpi4py-like ``comm``."""
    gathered = comm.gather(local_name2valcount)
    if comm.rank != 0:
        return {}
    sums, counts = defaultdict(float), defaultdict(float)
    for part in gathered:
        for name, (val, cnt) in part.items():
            try:
                val = float(val)
            except ValueError:
                continue
            sums[name] += val * cnt
            counts[name] += cnt
    return {n: sums[n] / counts[n] for n in sums}


def configure(dir=None, format_strs=None, comm=None, log_suffix="", append=False):
    """Configure the current logger (reference logger.py:448-481).

    ``append=True`` keeps existing ``log.txt``/``progress.csv`` content (resume).
    """
    if dir is None:
        dir = os.getenv("OPENAI_LOGDIR")
    if dir is None:
        dir = os.path.join(tempfile.gettempdir(),
                           datetime.datetime.now().strftime("openai-%Y-%m-%d-%H-%M-%S-%f"))
    assert isinstance(dir, str)
    dir = os.path.expanduser(dir)
    os.makedirs(dir, exist_ok=True)

    rank = _global_rank()
    if rank > 0:
        log_suffix = log_suffix + "-rank%03i" % rank
    if format_strs is None:
        env = "OPENAI_LOG_FORMAT" if rank == 0 else "OPENAI_LOG_FORMAT_MPI"
        format_strs = os.getenv(env, "stdout,log,csv" if rank == 0 else "log").split(",")
    formats = [make_output_format(f, dir, log_suffix, append=append) for f in format_strs if f]
    Logger.CURRENT = Logger(dir=dir, output_formats=formats, comm=comm)
    if formats:
        log("Logging to %s" % dir)


def _configure_default_logger():
    configure()
    Logger.DEFAULT = Logger.CURRENT


def reset():
    if Logger.CURRENT is not Logger.DEFAULT:
        Logger.CURRENT.close()
        Logger.CURRENT = Logger.DEFAULT
        log("Reset logger")


@contextmanager
def scoped_configure(dir=None, format_strs=None, comm=None):
    prev = Logger.CURRENT
    configure(dir=dir, format_strs=format_strs, comm=comm)
    try:
        yield
    finally:
        Logger.CURRENT.close()
        Logger.CURRENT = prev
