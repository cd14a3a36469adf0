"""Where do small library kernels come from?  For every dispatch whose name matches PATTERN in
a rocprofv3 kernel trace (csv), count the (previous, next) kernel names on the same queue -
the neighbouring native kernels identify the op that issued it.

    python tools/trace_neighbors.py gpurun_out/TRACE_DIR PATTERN [top]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main():
    d, pat = sys.argv[1], re.compile(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(p)))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append(r)
    pairs = collections.Counter()
    sizes = collections.Counter()
    n = 0
    for q, rs in byq.items():
        rs.sort(key=lambda r: int(r["Start_Timestamp"]))
        for i, r in enumerate(rs):
            if not pat.search(r["Kernel_Name"]):
                continue
            n += 1
            prev = short(rs[i - 1]["Kernel_Name"]) if i > 0 else "-"
            nxt = short(rs[i + 1]["Kernel_Name"]) if i + 1 < len(rs) else "-"
            pairs[(prev, nxt)] += 1
            sizes[r.get("Grid_Size_X", "?")] += 1
    print(f"# {n} dispatches matching {sys.argv[2]!r}; grid sizes: {dict(sizes.most_common(8))}")
    for (p, x), c in pairs.most_common(top):
        print(f"{c:6d}  after {p}\n        before {x}")


if __name__ == "__main__":
    main()
