"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (name incl. template args, truncated),
the per-dispatch mean of every collected counter.  usage: python profiles/pmc_summary.py <dir> [substr...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    subs = sys.argv[2:]
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        key = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    for key, cs in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_INSTS_VALU", 0))):
        n = len(disp[key])
        print(f"{key}  (dispatches {n})")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {v / n:16.1f}")


if __name__ == "__main__":
    main()
