"""
In-tree build of the native extension ``distributed_pipeline_amd/_C*.so``.

Compiles every ``csrc/*.hip`` kernel TU with ``hipcc --offload-arch=gfx950``
(no torch headers -> seconds per file) and the single ``csrc/bindings.cpp``
TU against the installed torch headers, then links one shared object next to
this file so it travels with the repository snapshot to the GPU box.

No hipify step is involved: sources are written for HIP/CDNA4 directly.
Object files are cached by content hash of (source, headers, flags), so a
rebuild only recompiles what changed.

usage: python -m distributed_pipeline_amd._build [--force] [--jobs N] [--debug]
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
ARCH = os.environ.get("DPA_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def _hipcc():
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"),
           os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def output_path():
    return os.path.join(HERE, EXT_NAME + _ext_suffix())


def _hash_files(paths, extra):
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode())
            h.update(f.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def _run(cmd):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("command failed (%d):\n%s\n%s" % (proc.returncode, " ".join(cmd), proc.stdout))
    return proc.stdout


def build(force=False, jobs=None, debug=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    kernels = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    binding = os.path.join(CSRC, "bindings.cpp")
    # host-side C++ (torch / c10d APIs): compiled with the binding flags
    host_cpp = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-Wno-unused-command-line-argument"] + opt
    tinc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    bind_flags = common + ["-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=" + EXT_NAME,
                           "-DTORCH_API_INCLUDE_EXTENSION_H", "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi,
                           "-I" + py_inc, "-Wno-deprecated-declarations"] + ["-I" + p for p in tinc]

    jobs_todo = []
    objects = []
    for src in kernels + [binding] + host_cpp:
        flags = bind_flags if (src == binding or src in host_cpp) else common
        key = _hash_files([src] + headers, " ".join(flags))
        obj = os.path.join(BUILD, os.path.basename(src) + "." + key + ".o")
        objects.append(obj)
        if force or not os.path.exists(obj):
            jobs_todo.append([_hipcc()] + flags + ["-I" + CSRC, "-c", src, "-o", obj])

    jobs = jobs or min(8, max(1, os.cpu_count() or 1))
    if jobs_todo:
        if verbose:
            print(f"[dpa build] compiling {len(jobs_todo)} TU(s) for {ARCH} with {jobs} jobs", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            for out in ex.map(_run, jobs_todo):
                if out.strip() and verbose:
                    print(out)

    target = output_path()
    link_key = _hash_files([], " ".join(objects))
    stamp = target + ".stamp"
    up_to_date = (os.path.exists(target) and os.path.exists(stamp)
                  and open(stamp).read().strip() == link_key)
    if force or not up_to_date:
        cmd = [_hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", target] + objects + [
            "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", "-lrccl", "-Wl,-rpath," + tlib]  # torch's own librccl: one RCCL per process
        _run(cmd)
        with open(stamp, "w") as f:
            f.write(link_key)
        if verbose:
            print(f"[dpa build] linked {target}", flush=True)
    # drop stale objects
    keep = set(objects)
    for o in glob.glob(os.path.join(BUILD, "*.o")):
        if o not in keep:
            os.remove(o)
    return target


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    print(build(force=a.force, jobs=a.jobs, debug=a.debug))


if __name__ == "__main__":
    sys.exit(main())
