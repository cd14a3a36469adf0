"""bench.py with one engine attribute patched, for in-process A/Bs of settings that are not
environment knobs.  Usage:

    python tools/probes/bench_patched.py --set ops.nn._WgradDeferral.grouped=False -- [bench.py args]

``--set MODULE.CLASS.ATTR=VALUE`` (repeatable; VALUE through ast.literal_eval) patches
``distributed_pipeline_amd.<MODULE>``'s attribute before bench.py runs in this process."""
import ast
import importlib
import os
import runpy
import sys


def main():
    argv = sys.argv[1:]
    sets = []
    while argv and argv[0] == "--set":
        sets.append(argv[1])
        argv = argv[2:]
    if argv and argv[0] == "--":
        argv = argv[1:]
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, root)
    for s in sets:
        path, val = s.split("=", 1)
        mod, cls, attr = path.rsplit(".", 2)
        obj = getattr(importlib.import_module("distributed_pipeline_amd." + mod), cls)
        setattr(obj, attr, ast.literal_eval(val))
        print(f"[bench_patched] {path} = {val!r}", flush=True)
    sys.argv = [os.path.join(root, "bench.py")] + argv
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
