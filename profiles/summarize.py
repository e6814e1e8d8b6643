"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time (per-call average in us)."""
import csv
import sys


def main(path, top=25, steps=1):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:9.2f} ms {float(r['Percentage']):6.2f}% "
              f"n={int(r['Calls']) // steps:>6} avg={float(r['AverageNs']) / 1e3:9.2f}us  {r['Name'][:100]}")
    print(f"total kernel ms per step: {tot / 1e6 / steps:.1f}")


if __name__ == "__main__":
    main(sys.argv[1], steps=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
