# Host-side profile (cProfile, backward on the calling thread) of the reference 32 x 64 schedule.
set -o pipefail
mkdir -p gpurun_out/hostprof
timeout -k 10 400 python tools/host_prof.py gpurun_out/hostprof/ref.prof --steps 1 --warmup 1 --ref-steps 4 --json-out gpurun_out/hostprof/b.json > gpurun_out/hostprof/b.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/hostprof/top.txt
import pstats
p = pstats.Stats("gpurun_out/hostprof/ref.prof")
p.sort_stats("tottime").print_stats(70)
p.sort_stats("cumulative").print_stats(120)
PY
