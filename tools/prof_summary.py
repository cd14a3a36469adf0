"""Summarise a rocprofv3 kernel trace: top kernels by total time.

Accepts a directory holding either ``*kernel_stats.csv`` (``--stats`` CSV output)
or ``*_results.db`` (rocpd SQLite output), or one such file.

    python tools/prof_summary.py gpurun_out/prof5 [top] [steps] [--by-grid]

``steps``: divide totals by this many optimizer steps (ms/step column).
``--by-grid``: split each kernel by its grid size (tells GEMM shapes apart).
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def _rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield r["Name"], None, float(r["TotalDurationNs"]), int(r["Calls"])


def _rows_db(path):
    con = sqlite3.connect(path)
    for name, gx, dur in con.execute("select name, grid_x, duration from kernels"):
        yield name, gx, float(dur), 1


def load(path, by_grid=False):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*_results.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        path = (dbs or csvs)[0]
    it = _rows_db(path) if path.endswith(".db") else _rows_csv(path)
    agg = collections.defaultdict(lambda: [0.0, 0])
    for name, grid, ns, calls in it:
        key = (name, grid if by_grid else None)
        agg[key][0] += ns
        agg[key][1] += calls
    return path, agg


def main(argv):
    by_grid = "--by-grid" in argv
    argv = [a for a in argv if a != "--by-grid"]
    path = argv[0]
    top = int(argv[1]) if len(argv) > 1 else 30
    steps = int(argv[2]) if len(argv) > 2 else None
    src, agg = load(path, by_grid)
    tot = sum(v[0] for v in agg.values())
    per = f" = {tot / 1e6 / steps:.2f} ms/step over {steps} steps" if steps else ""
    print(f"# {src}\n# total kernel time {tot / 1e6:.2f} ms{per}")
    for (name, grid), (ns, calls) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        ps = f"{ns / 1e6 / steps:8.2f} ms/step" if steps else ""
        g = f" grid={grid}" if grid is not None else ""
        print(f"{ns / 1e6:9.2f} ms {100 * ns / tot:6.2f}% {ps} n={calls:>6}{g} {name[:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
