#!/bin/bash
# Host ASan/UBSan run of the native DDP engine tests on CPU (gloo ranks).
set -eo pipefail
cd "$(dirname "$0")/.."
python tools/asan_build.py
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0,abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  DPA_EXT=_C_asan python -m pytest tests/test_ddp_engine.py -x -q -p no:cacheprovider "$@" || { rc=$?; rm -f distributed_pipeline_amd/_C_asan*.so; exit $rc; }
rm -f distributed_pipeline_amd/_C_asan*.so
