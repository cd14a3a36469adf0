"""Stream concurrency in a rocprofv3 kernel trace.

    python tools/trace_overlap.py gpurun_out/gab2/tr/run_kernel_trace.csv [--last-ms 600] [--gap-ms 50]

Splits the trace into bursts (idle gaps longer than ``--gap-ms`` end a burst) and reports, per
burst: wall time, the sum of kernel durations, their ratio (> 1 = kernels of different queues
ran concurrently), the busy union, and per-queue kernel counts and busy time.  Used to check
whether a replayed HIP graph keeps the overlapped micro-batch schedule's streams concurrent
(utils/trainer.py ``_forward_backward_overlapped``) or serialises them.
"""
import argparse
import csv
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         r["Kernel_Name"][:60]))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def bursts(rows, gap_ns):
    out, cur, last_end = [], [], None
    for r in rows:
        if last_end is not None and r[0] - last_end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(r)
        last_end = r[1] if last_end is None else max(last_end, r[1])
    if cur:
        out.append(cur)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--min-ms", type=float, default=20.0, help="skip bursts shorter than this")
    a = ap.parse_args()
    rows = load(a.trace)
    for i, b in enumerate(bursts(rows, int(a.gap_ms * 1e6))):
        wall = (max(r[1] for r in b) - b[0][0]) / 1e6
        if wall < a.min_ms:
            continue
        ksum = sum(r[1] - r[0] for r in b) / 1e6
        busy = union([(r[0], r[1]) for r in b]) / 1e6
        perq = defaultdict(list)
        for r in b:
            perq[r[2]].append((r[0], r[1]))
        qs = ", ".join(f"q{q}: n={len(v)} busy={union(v) / 1e6:.1f} ms" for q, v in sorted(perq.items()))
        print(f"burst {i}: wall {wall:.1f} ms, kernel sum {ksum:.1f} ms (x{ksum / wall:.2f}), "
              f"busy union {busy:.1f} ms, {len(b)} kernels; {qs}")


if __name__ == "__main__":
    main()
