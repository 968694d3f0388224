"""Summarise rocprofv3 CSV output (kernel_stats / counter_collection) to markdown.

    python -m multidisttorch_amd.obs.summarize_prof <rocprof_dir> [--steps N] [--top 15]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def kernel_stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        return []
    rows = list(csv.DictReader(open(f[0])))
    return rows


def counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=None, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args(argv)
    rows = kernel_stats(a.dir)
    if rows:
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print(f"| kernel | calls | avg us | total ms | % |{' us/step |' if a.steps else ''}")
        print(f"|---|---|---|---|---|{'---|' if a.steps else ''}")
        for r in rows[: a.top]:
            name = r["Name"].split("(")[0][:70]
            line = (f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                    f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
            if a.steps:
                line += f" {float(r['TotalDurationNs'])/1e3/a.steps:.2f} |"
            print(line)
        print(f"\nTotal GPU kernel time: {tot/1e6:.3f} ms")
    c = counters(a.dir)
    if c:
        print("\n| kernel | counter | mean per dispatch |\n|---|---|---|")
        for (k, n), v in sorted(c.items()):
            if "mdt" in k:
                print(f"| `{k}` | {n} | {sum(v)/len(v):.0f} |")


if __name__ == "__main__":
    main()
