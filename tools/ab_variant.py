"""Build an A/B variant of the extension with some csrc/ files taken from another git revision.

    python tools/ab_variant.py REV csrc/attention.hip [csrc/norm.hip ...]   # -> distributed_pipeline_amd/_C_ab*.so
    python tools/ab_variant.py REV                                          # the whole csrc/ of REV

With files named, every other translation unit is the current tree's (the named files must keep
the launchers.h interface); with none, every source and header comes from REV.  Same flags as
distributed_pipeline_amd/_build.py; the binding is recompiled with TORCH_EXTENSION_NAME=_C_ab.
Select it at run time with DPA_EXT=_C_ab, so one process pair on one GPU box times old vs new
kernels back to back.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from distributed_pipeline_amd import _build as B  # noqa: E402


def main(argv):
    rev, files = argv[0], argv[1:]
    work = os.path.join(B.BUILD, "ab")
    os.makedirs(work, exist_ok=True)
    csrc = B.CSRC
    if not files:  # the whole native tree of REV
        csrc = os.path.join(work, "csrc")
        os.makedirs(os.path.join(csrc, "comm"), exist_ok=True)
        os.makedirs(os.path.join(csrc, "runtime"), exist_ok=True)
        names = subprocess.check_output(["git", "-C", HERE, "ls-tree", "-r", "--name-only", rev,
                                         "distributed_pipeline_amd/csrc"], text=True).split()
        for n in names:
            dst = os.path.join(csrc, os.path.relpath(n, "distributed_pipeline_amd/csrc"))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            with open(dst, "w") as fh:
                fh.write(subprocess.check_output(["git", "-C", HERE, "show", f"{rev}:{n}"], text=True))
    tinc, tlib, abi = B._torch_paths()
    import sysconfig
    common = ["-std=c++17", "-fPIC", "--offload-arch=" + B.ARCH, "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-Wno-unused-command-line-argument", "-O3", "-I" + csrc]
    bind = common + ["-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C_ab", "-DTORCH_API_INCLUDE_EXTENSION_H",
                     "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi, "-I" + sysconfig.get_paths()["include"],
                     "-Wno-deprecated-declarations"] + ["-I" + p for p in tinc]
    swapped = {os.path.basename(f) for f in files}
    objs = []
    for f in files:
        src = os.path.join(work, os.path.basename(f))
        with open(src, "w") as fh:
            fh.write(subprocess.check_output(["git", "-C", HERE, "show", f"{rev}:distributed_pipeline_amd/{f}"],
                                             text=True))
        obj = src + ".o"
        B._run([B._hipcc()] + common + ["-c", src, "-o", obj])
        objs.append(obj)
    for src in sorted(glob.glob(os.path.join(csrc, "*.hip"))):
        if os.path.basename(src) in swapped:
            continue
        obj = os.path.join(work, os.path.basename(src) + ".cur.o")
        B._run([B._hipcc()] + common + ["-c", src, "-o", obj])
        objs.append(obj)
    for src in [os.path.join(csrc, "bindings.cpp")] + sorted(glob.glob(os.path.join(csrc, "comm", "*.cpp"))
                                                          + glob.glob(os.path.join(csrc, "runtime", "*.cpp"))):
        obj = os.path.join(work, os.path.basename(src) + ".ab.o")
        B._run([B._hipcc()] + bind + ["-c", src, "-o", obj])
        objs.append(obj)
    target = os.path.join(HERE, "distributed_pipeline_amd", "_C_ab" + B._ext_suffix())
    B._run([B._hipcc(), "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-o", target] + objs + [
        "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lrccl",
        "-Wl,-rpath," + tlib])
    print(target)


if __name__ == "__main__":
    main(sys.argv[1:])
