"""Loader for the in-tree native extension (``distributed_pipeline_amd/_C*.so``).

Policy: on a machine with a visible HIP device the extension is REQUIRED -
every op that has a gfx950 kernel runs it, and a missing/broken build raises
immediately instead of silently falling back to eager PyTorch.  On CPU-only
hosts (unit tests) ops use their PyTorch reference implementations.

Debug mode: ``DPA_SYNC_CHECK=1`` returns a proxy of the module whose
functions synchronise the device after every native call and re-raise any HIP
error together with the op name and its tensor shapes/dtypes, so an
asynchronous fault (out-of-bounds access, bad launch) is attributed to the
kernel that caused it rather than to whatever op synchronises next.  The cost
is one device sync per op; use it for debugging only.
"""
import importlib
import os

import torch

_EXT = None
_ERR = None


def _describe(args):
    out = []
    for a in args:
        if isinstance(a, torch.Tensor):
            out.append(f"Tensor{tuple(a.shape)}:{str(a.dtype).replace('torch.', '')}@{a.device}")
        else:
            out.append(type(a).__name__ if not isinstance(a, (int, float, bool)) else repr(a))
    return ", ".join(out)


class _SyncChecked:
    """Module proxy: every pybind function call is followed by a device sync."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        attr = getattr(self._mod, name)
        if type(attr).__name__ != "builtin_function_or_method":
            return attr

        def checked(*args, **kwargs):
            try:
                out = attr(*args, **kwargs)
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
            except Exception as exc:  # noqa: BLE001
                raise RuntimeError(f"[DPA_SYNC_CHECK] native op {name}({_describe(args)}) failed: "
                                   f"{exc}") from exc
            return out

        checked.__name__ = name
        return checked


_NATIVE_ENABLED = True


def set_native_enabled(flag):
    """``use_hip_kernels`` setting: False routes every op to its PyTorch reference path
    (the eager ATen / hipBLASLt implementation) even on a GPU - an A/B and debugging
    switch, never the default."""
    global _NATIVE_ENABLED
    _NATIVE_ENABLED = bool(flag)


def gpu_present():
    return torch.cuda.is_available()


_REQUIRED = None  # default of get_ext(required=None), evaluated once per process


def get_ext(required=None):
    """Return the ``_C`` module.  ``required`` defaults to "a GPU is present".

    Called once or more per op on the hot path (a reference-schedule micro-batch makes ~200
    calls): once loaded, the common case returns before any device query or env read."""
    global _EXT, _ERR, _REQUIRED
    if required is None and _EXT is not None:
        return _EXT if _NATIVE_ENABLED else None
    if not _NATIVE_ENABLED and not required:
        return None
    if _EXT is None and _ERR is None:
        try:
            # DPA_EXT selects an alternative build of the same sources, e.g. the
            # host-ASan build ``_C_asan`` of tools/asan_build.py
            _EXT = importlib.import_module("distributed_pipeline_amd." + os.environ.get("DPA_EXT", "_C"))
            if os.environ.get("DPA_SYNC_CHECK", "0") == "1":
                _EXT = _SyncChecked(_EXT)
        except Exception as exc:  # noqa: BLE001
            _ERR = exc
    if required is None:
        if _REQUIRED is None:
            _REQUIRED = gpu_present() and os.environ.get("DPA_ALLOW_NO_EXT", "0") != "1"
        required = _REQUIRED
    if _EXT is None and required:
        raise RuntimeError(
            "distributed_pipeline_amd native extension is not built/loadable "
            f"({_ERR!r}); run `python -m distributed_pipeline_amd._build`") from _ERR
    return _EXT


def use_native(t):
    """True when tensor ``t`` should go through a HIP kernel."""
    return t.is_cuda and get_ext() is not None
