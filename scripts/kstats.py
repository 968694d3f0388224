"""Summarise a rocprofv3 kernel_trace.csv: per-kernel time over the last N dispatches window.

usage: python scripts/kstats.py <kernel_trace.csv> [steps_in_window]
Prints average duration per call and calls, sorted by total time (only kernels
from the mdt namespace and rocclr copies; torch setup kernels are excluded).
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    n = r["Kernel_Name"]
    if "at::native" in n:
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[n] += dur
    cnt[n] += 1
allt = sum(tot.values())
for n in sorted(tot, key=lambda k: -tot[k])[:40]:
    print(f"{tot[n]:10.1f} us  calls={cnt[n]:5d}  avg={tot[n] / cnt[n]:8.2f} us  {n[:120]}")
print("total", round(allt, 1), "us")
