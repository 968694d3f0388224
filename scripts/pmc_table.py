"""Aggregate rocprofv3 counter_collection.csv files: mean counter value per kernel."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "at::native" in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in acc for c in acc[k]})
print("| kernel | " + " | ".join(names) + " |")
print("|---" * (len(names) + 1) + "|")
for k in sorted(acc):
    vals = [acc[k][c] for c in names]
    cells = [f"{sum(v) / len(v):.3g}" if v else "" for v in vals]
    short = k.replace("mdt::", "").replace("(mdt::IgArgs)", "").replace("(mdt::WgArgs)", "")[:70]
    print(f"| `{short}` | " + " | ".join(cells) + " |")
