#!/usr/bin/env python3
"""Per-kernel MFMA utilisation and HBM traffic from rocprofv3 counter passes.

    python scripts/pmc_roofline.py SQ_PASS.csv FETCH_PASS.csv WRITE_PASS.csv

SQ_PASS holds SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA,
SQ_INSTS_VALU, GRBM_GUI_ACTIVE; the other two FETCH_SIZE / WRITE_SIZE (KB),
each its own pass. Per kernel (mean over dispatches, torch kernels skipped):
duration under the counters, MFMA busy as a fraction of the chip's SIMD-cycles
(SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x 2.4 GHz); GRBM_GUI_ACTIVE
is summed over the XCDs, so the duration is the clock base), the VALU:MFMA
instruction ratio, fabric bytes fetched / written and their rate. Durations
are inflated by the counter collection (~1 us per launch).
"""
import csv
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    seen = set()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "at::native" in k or "anonymous namespace" in k or "rocclr" in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (r["Dispatch_Id"], k)
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return acc, dur


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def short(k):
    k = k.replace("mdt::", "").replace("void ", "")
    for t in ("(JobPack)", "(DcArgs)", "(DwArgs)", "(IgArgs)", "(WgArgs)", "(ThinConvArgs)", "(ThinTconvArgs)"):
        k = k.replace(t, "")
    return k[:90]


def main():
    sq, dur = load(sys.argv[1])
    fe, _ = load(sys.argv[2]) if len(sys.argv) > 2 else ({}, {})
    wr, _ = load(sys.argv[3]) if len(sys.argv) > 3 else ({}, {})
    rows = []
    for k in sq:
        c = sq[k]
        d = mean(dur[k])
        busy = mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        mf = mean(c.get("SQ_INSTS_MFMA", []))
        va = mean(c.get("SQ_INSTS_VALU", []))
        f = mean(fe.get(k, {}).get("FETCH_SIZE", [])) / 1e3 if k in fe else float("nan")
        w = mean(wr.get(k, {}).get("WRITE_SIZE", [])) / 1e3 if k in wr else float("nan")
        rows.append((d * len(dur[k]), k, d, 100 * busy / (1024 * d * 2400.0) if d else float("nan"),
                     va / mf if mf else float("inf"), f, w, (f + w) / d if d else float("nan")))
    rows.sort(reverse=True)
    print("| kernel | us | MFMA busy % of SIMD-cycles | VALU:MFMA instr | fetch MB | write MB | fabric TB/s |")
    print("|---|---|---|---|---|---|---|")
    for _, k, d, b, r, f, w, bw in rows:
        rr = "-" if r == float("inf") else f"{r:.1f}"
        print(f"| `{short(k)}` | {d:.1f} | {b:.1f} | {rr} | {f:.1f} | {w:.1f} | {bw:.2f} |")


if __name__ == "__main__":
    main()
