"""Host-side AddressSanitizer build of the native extension.

Builds ``distributed_pipeline_amd/_C_asan*.so`` from the same sources as
``_build.py`` with ASan + UBSan on the HOST code only (the C++ bucket reducer,
the pybind bindings and every kernel launcher); device code is compiled
exactly as in the normal build.  Run the CPU engine tests against it with

    tools/asan_check.sh

which preloads the clang ASan runtime into python and selects the build with
``DPA_EXT=_C_asan``.  This checks the host paths that the gloo-backed CPU
tests drive (bucket planning, hook bookkeeping, in-place flat all-reduce,
bf16 wire staging) for heap/stack overflows, use-after-free and UB.
"""
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from distributed_pipeline_amd import _build as B  # noqa: E402

HOST_SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
            "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]


def build():
    out_dir = os.path.join(B.HERE, "build_asan")
    os.makedirs(out_dir, exist_ok=True)
    name = "_C_asan"
    tinc, tlib, abi = B._torch_paths()
    import sysconfig
    common = ["-std=c++17", "-fPIC", "--offload-arch=" + B.ARCH, "-O1", "-g",
              "-Wno-unused-result", "-Wno-unused-command-line-argument"] + HOST_SAN
    bind = common + ["-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=" + name, "-DTORCH_API_INCLUDE_EXTENSION_H",
                     "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi, "-I" + sysconfig.get_paths()["include"],
                     "-Wno-deprecated-declarations"] + ["-I" + p for p in tinc]
    srcs = sorted(glob.glob(os.path.join(B.CSRC, "*.hip")))
    host = [os.path.join(B.CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(B.CSRC, "comm", "*.cpp")))
    import concurrent.futures as cf
    jobs, objs = [], []
    for src in srcs + host:
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        flags = bind if src in host else common
        jobs.append([B._hipcc()] + flags + ["-I" + B.CSRC, "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(B._run, jobs))
    target = os.path.join(B.HERE, name + B._ext_suffix())
    B._run([B._hipcc(), "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-fsanitize=address,undefined",
            "-fno-gpu-sanitize", "-shared-libsan", "-o", target] + objs +
           ["-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-Wl,-rpath," + tlib])
    print(target)
    return target


if __name__ == "__main__":
    build()
