"""Per-launch HBM traffic of the vocoder conv kernel from two rocprofv3 PMC passes.

FETCH_SIZE and WRITE_SIZE (KiB per dispatch) come from separate passes (they do not fit in one
TCC pass on gfx950).  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section), gfx950 FETCH_SIZE
reports half the bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  Only the second half of the ``igemm_kernel`` dispatches (the second forward
of profiles/pmc_vocoder.py) is averaged.

usage: python profiles/traffic.py <fetch_dir> <write_dir>  -> JSON on stdout
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "igemm_kernel" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    ids = sorted(vals)
    ids = ids[len(ids) // 2:]
    return [vals[i] for i in ids]


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    n = min(len(fetch), len(write))
    fetch_b = [2 * 1024 * v for v in fetch[:n]]  # KiB -> bytes, x2 gfx950 correction
    write_b = [1024 * v for v in write[:n]]
    out = {
        "kernel": "igemm_kernel (BigVGAN convs, second of two C3 vocoder forwards)",
        "dispatches": n,
        "fetch_bytes_per_launch": sum(fetch_b) / n,
        "write_bytes_per_launch": sum(write_b) / n,
        "igemm_bytes_per_launch": (sum(fetch_b) + sum(write_b)) / n,
        "correction": "FETCH_SIZE x2 (gfx950 coalesced-read undercount); KiB -> bytes",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
