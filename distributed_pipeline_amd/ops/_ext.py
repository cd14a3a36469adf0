"""Loader for the in-tree native extension (``distributed_pipeline_amd/_C*.so``).

Policy: on a machine with a visible HIP device the extension is REQUIRED -
every op that has a gfx950 kernel runs it, and a missing/broken build raises
immediately instead of silently falling back to eager PyTorch.  On CPU-only
hosts (unit tests) ops use their PyTorch reference implementations.
"""
import importlib
import os

import torch

_EXT = None
_ERR = None


def gpu_present():
    return torch.cuda.is_available()


def get_ext(required=None):
    """Return the ``_C`` module.  ``required`` defaults to "a GPU is present"."""
    global _EXT, _ERR
    if _EXT is None and _ERR is None:
        try:
            _EXT = importlib.import_module("distributed_pipeline_amd._C")
        except Exception as exc:  # noqa: BLE001
            _ERR = exc
    if required is None:
        required = gpu_present() and os.environ.get("DPA_ALLOW_NO_EXT", "0") != "1"
    if _EXT is None and required:
        raise RuntimeError(
            "distributed_pipeline_amd native extension is not built/loadable "
            f"({_ERR!r}); run `python -m distributed_pipeline_amd._build`") from _ERR
    return _EXT


def use_native(t):
    """True when tensor ``t`` should go through a HIP kernel."""
    return t.is_cuda and get_ext() is not None
