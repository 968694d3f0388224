"""Per-position kernel timeline of a repeating step from a rocprofv3 kernel_trace.csv.

usage: python scripts/ktimeline.py <kernel_trace.csv> <first-kernel-substring> [skip_steps]
Splits the dispatch stream into steps at every kernel whose name contains the
marker, then reports for each position in the step the median duration and the
median gap from the previous kernel's end (launch/boundary cost as seen on the
device), plus the median step span.
"""
import csv
import statistics as stt
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "at::native" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 5
steps, cur = [], None
for r in rows:
    if marker in r["Kernel_Name"]:
        if cur:
            steps.append(cur)
        cur = []
    if cur is not None:
        cur.append(r)
steps = steps[skip:]
L = stt.mode([len(s) for s in steps])
steps = [s for s in steps if len(s) == L]
print(f"steps={len(steps)} kernels/step={L}")
spans = []
tot_d = tot_g = 0.0
for i in range(L):
    ds = [(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"])) / 1e3 for s in steps]
    gs = [(int(s[i]["Start_Timestamp"]) - int(s[i - 1]["End_Timestamp"])) / 1e3 for s in steps] if i else [0.0]
    d, g = stt.median(ds), stt.median(gs)
    tot_d += d
    tot_g += g
    name = steps[0][i]["Kernel_Name"]
    name = name.replace("void ", "").replace("mdt::", "")[:90]
    print(f"{i:3d} gap {g:6.2f}  dur {d:7.2f}  {name}")
for s in steps[:-1]:
    pass
spans = [(int(b[0]["Start_Timestamp"]) - int(a[0]["Start_Timestamp"])) / 1e3 for a, b in zip(steps, steps[1:])]
print(f"sum dur {tot_d:.1f} us, sum gaps {tot_g:.1f} us, median step period {stt.median(spans):.1f} us")
