"""Which launches neighbour the __amd_rocclr_copyBuffer dispatches of a bench run (rocprofv3
--kernel-trace CSV): counts of (previous kernel, next kernel) name pairs around each copy."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"][:70] for r in rows]
pairs = collections.Counter()
for i, n in enumerate(names):
    if "copyBuffer" in n:
        prev = names[i - 1] if i else "-"
        nxt = names[i + 1] if i + 1 < len(names) else "-"
        pairs[(prev, nxt)] += 1
for (p, q), c in pairs.most_common(15):
    print(f"{c:6d}  after {p}  |  before {q}")
print("total copies", sum(pairs.values()), "of", len(rows), "dispatches")
