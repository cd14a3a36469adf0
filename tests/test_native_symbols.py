"""The in-tree extension must load against the HIP runtime torch ships (the GPU boxes load
torch's libamdhip64 first): every hip* symbol _C imports has to be exported by it.  A symbol
only /opt/rocm's newer runtime has (e.g. hipStreamGetId, hip_7.1) links fine here and fails
to import on the box."""
import os
import shutil
import subprocess

import pytest
import torch


def _syms(path, undefined):
    out = subprocess.run(["nm", "-D", path], capture_output=True, text=True, check=True).stdout
    names = set()
    for line in out.splitlines():
        parts = line.split()
        if undefined and len(parts) == 2 and parts[0] == "U":
            names.add(parts[1].split("@")[0])
        elif not undefined and len(parts) == 3 and parts[1] in ("T", "W"):
            names.add(parts[2].split("@")[0])
    return names


def test_extension_hip_symbols_exist_in_torch_runtime():
    from distributed_pipeline_amd import _build
    so = _build.output_path()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if not (os.path.exists(so) and os.path.exists(lib) and shutil.which("nm")):
        pytest.skip("extension, torch HIP runtime or nm not available")
    need = {s for s in _syms(so, True) if s.startswith("hip")}
    have = _syms(lib, False)
    assert need and not (need - have), sorted(need - have)
