"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import glob
import sys


def main(path, top=30, steps=None):
    files = glob.glob(path + "/**/*kernel_stats.csv", recursive=True) if not path.endswith(".csv") else [path]
    rows = list(csv.DictReader(open(files[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {files[0]}\n# total kernel time {tot / 1e6:.2f} ms" + (f" ({tot / 1e6 / steps:.2f} ms/step over {steps} steps)" if steps else ""))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>6} {r['Name'][:120]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30,
         int(sys.argv[3]) if len(sys.argv) > 3 else None)
