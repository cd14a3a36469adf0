"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (top by
SQ_BUSY_CYCLES), the sum of every collected counter plus derived ratios
(MFMA busy share of SQ busy cycles, LDS bank-conflict cycles per LDS instruction).

    python tools/pmc_summary.py <dir-with-*counter_collection.csv> [top]
"""
import collections
import csv
import glob
import os
import sys


def main(argv):
    path = argv[0]
    top = int(argv[1]) if len(argv) > 1 else 15
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                           recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or "?"
            agg[name[:90]][r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"# {files}")
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0.0))[:top]
    for name, c in rows:
        busy = c.get("SQ_BUSY_CYCLES", 0.0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        lds = c.get("SQ_INSTS_LDS", 0.0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        extra = {k: f"{v:.3g}" for k, v in sorted(c.items())}
        print(f"{name}\n    mfma_busy/sq_busy={mf / busy if busy else 0:.3f} "
              f"lds_conflict_cycles_per_lds_inst={bc / lds if lds else 0:.3f} {extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
