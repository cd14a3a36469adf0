"""Parametrised GPU runner: one ``gpurun`` call = one list of steps, each under its own
time limit; the first failing step ends the call (nothing is retried).

    /usr/local/graft/bin/gpurun --timeout 900 -- 'python tools/gpu/run.py STEP [STEP ...]'

Steps (``:``-separated fields; ``,`` separates extra command-line arguments):
    env:VAR=VAL                 set an environment variable for the following steps
    tests[:FILES]               pytest -m gpu (FILES: comma-separated test files, default all)
    tests?[:FILES]              the same, but failing tests (pytest status 1) do not end the call
    smoke                       __graft_entry__.smoke()
    bench:NAME[:ARGS]           python bench.py ARGS -> gpurun_out/NAME.{log,json}
    prof:NAME[:ARGS]            rocprofv3 --kernel-trace --stats of a 3-step bench (+ARGS) ->
                                gpurun_out/NAME/summary.txt (tools/prof_summary.py)
    ab:VAR:A:B[:REPS[:ARGS]]    interleaved headline benches with VAR=A / VAR=B -> gpurun_out/ab_VAR.txt
    py:NAME:SCRIPT[:ARGS]       python SCRIPT ARGS -> gpurun_out/NAME.log
    trace:NAME:SCRIPT[:ARGS]    rocprofv3 --kernel-trace (csv) of python SCRIPT ARGS -> gpurun_out/NAME/
    profpy:NAME:SCRIPT[:ARGS[:N]]  rocprofv3 --kernel-trace --stats of python SCRIPT ARGS, summarised per N steps

This process never touches the GPU itself (it only starts children), so the children
may exec freely.
"""
import json
import os
import subprocess
import sys
import time

OUT = "gpurun_out"


def _run(cmd, log, limit, env=None, ok_codes=(0,)):
    """Run one step; any exit status outside ok_codes ends the call (faults, aborts and time
    limits always do: only pytest's "tests failed" status 1 may be tolerated)."""
    t0 = time.time()
    print(f"[run] {' '.join(cmd)}  (limit {limit}s) -> {log}", flush=True)
    with open(log, "w") as f:
        p = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                           env=env)
    print(f"[run] exit {p.returncode} after {time.time() - t0:.1f}s", flush=True)
    if p.returncode not in ok_codes:
        with open(log) as f:
            tail = f.read()[-3000:]
        print(tail, flush=True)
        sys.exit(p.returncode)


def _bench_ms(path):
    """headline ms/step, plus the reference schedule's when it ran"""
    with open(path) as f:
        d = json.load(f)
    r = (d.get("reference_schedule") or {}).get("ms_per_step")
    return f"{d['ms_per_step']}" + (f" (reference schedule {r})" if r else "")


def main(steps):
    os.makedirs(OUT, exist_ok=True)
    ntest = [0]
    env = dict(os.environ)
    # tools/*.py scripts import the package from the repository root
    env["PYTHONPATH"] = os.getcwd() + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    for st in steps:
        f = st.split(":")
        kind = f[0]
        if kind == "env":
            k, v = f[1].split("=", 1)
            env[k] = v
            print(f"[run] env {k}={v}", flush=True)
        elif kind in ("tests", "tests?"):  # tests?: a failing test (pytest status 1) does not end the call
            files = [os.path.join("tests", x) for x in f[1].split(",")] if len(f) > 1 and f[1] else ["tests"]
            ntest[0] += 1
            log = os.path.join(OUT, "gputests.log" if ntest[0] == 1 else f"gputests_{ntest[0]}.log")
            _run([sys.executable, "-u", "-m", "pytest", "-m", "gpu", "-x", "-v", "--timeout", "120",
                  "--timeout-method", "thread"] + files, log, 1000, env,
                 ok_codes=(0, 1) if kind == "tests?" else (0,))
            with open(log) as fh:
                print(fh.read().strip().splitlines()[-1], flush=True)
        elif kind == "smoke":
            _run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], os.path.join(OUT, "smoke.log"),
                 240, env)
        elif kind == "bench":
            name = f[1]
            args = f[2].split(",") if len(f) > 2 and f[2] else []
            js = os.path.join(OUT, name + ".json")
            _run([sys.executable, "-u", "bench.py", "--json-out", js] + args, os.path.join(OUT, name + ".log"), 600,
                 env)
            with open(js) as fh:
                d = json.load(fh)
            print(f"[run] {name}: {d['ms_per_step']} ms/step; reference schedule "
                  f"{(d.get('reference_schedule') or {}).get('ms_per_step')}", flush=True)
        elif kind == "prof":
            name = f[1]
            args = f[2].split(",") if len(f) > 2 and f[2] else []
            d = os.path.join(OUT, name)
            os.makedirs(d, exist_ok=True)
            steps_n = "3"
            _run(["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run", "--", sys.executable, "bench.py",
                  "--steps", steps_n, "--warmup", "1", "--ref-steps", "0", "--comm-probe", "0"] + args,
                 os.path.join(d, "prof.log"), 600, dict(env, TMPDIR="/tmp"))
            # kernel stats of warmup + timed steps: the summary divides by their count
            _run([sys.executable, "tools/prof_summary.py", d, "40", str(int(steps_n) + 1)],
                 os.path.join(d, "summary.txt"), 120, env)
            with open(os.path.join(d, "summary.txt")) as fh:
                print(fh.read()[:4000], flush=True)
            # the trace database runs to tens of MB: only the summary comes back (gpurun's 64 MiB cap)
            for f_ in os.listdir(d):
                if f_.endswith(".db"):
                    os.remove(os.path.join(d, f_))
        elif kind == "profpy":  # profpy:NAME:SCRIPT[:ARGS[:STEPS]] - kernel stats of a python script
            name, script = f[1], f[2]
            args = f[3].split(",") if len(f) > 3 and f[3] else []
            nsteps = f[4] if len(f) > 4 and f[4] else "1"
            d = os.path.join(OUT, name)
            os.makedirs(d, exist_ok=True)
            _run(["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run", "--", sys.executable, "-u", script]
                 + args, os.path.join(d, "prof.log"), 600, dict(env, TMPDIR="/tmp"))
            _run([sys.executable, "tools/prof_summary.py", d, "40", nsteps], os.path.join(d, "summary.txt"), 120, env)
            with open(os.path.join(d, "summary.txt")) as fh:
                print(fh.read()[:3000], flush=True)
            for f_ in os.listdir(d):
                if f_.endswith(".db"):
                    os.remove(os.path.join(d, f_))
        elif kind == "ab":
            var, a, b = f[1], f[2], f[3]
            reps = int(f[4]) if len(f) > 4 and f[4] else 2
            args = f[5].split(",") if len(f) > 5 and f[5] else ["--ref-steps", "0"]
            lines = []
            for i in range(reps):
                for v in (a, b):
                    js = os.path.join(OUT, f"ab_{var}_{v}_{i}.json")
                    _run([sys.executable, "-u", "bench.py", "--steps", "10", "--warmup", "3", "--json-out", js] + args,
                         os.path.join(OUT, f"ab_{var}_{v}_{i}.log"), 600, dict(env, **{var: v}))
                    line = f"{var}={v} rep {i}: {_bench_ms(js)} ms/step"
                    print("[run] " + line, flush=True)
                    lines.append(line)
            with open(os.path.join(OUT, f"ab_{var}.txt"), "a") as fh:
                fh.write("\n".join(lines) + "\n")
        elif kind == "trace":  # trace:NAME:SCRIPT[:ARGS] - a kernel trace (csv) of a python script
            name, script = f[1], f[2]
            args = f[3].split(",") if len(f) > 3 and f[3] else []
            d = os.path.join(OUT, name)
            os.makedirs(d, exist_ok=True)
            _run(["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", name, "--",
                  sys.executable, "-u", script] + args, os.path.join(d, "trace.log"), 600,
                 dict(env, TMPDIR="/tmp", SQ_OUT=os.path.join(d, "order.json")))
        elif kind == "py":
            name, script = f[1], f[2]
            args = f[3].split(",") if len(f) > 3 and f[3] else []
            _run([sys.executable, "-u", script] + args, os.path.join(OUT, name + ".log"), 900, env)
            with open(os.path.join(OUT, name + ".log")) as fh:
                print(fh.read()[-3000:], flush=True)
        else:
            sys.exit(f"unknown step {st!r}")


if __name__ == "__main__":
    main(sys.argv[1:])
