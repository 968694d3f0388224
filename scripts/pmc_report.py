"""Per-kernel PMC report from rocprofv3 counter_collection CSVs (several passes).

usage: python scripts/pmc_report.py "<glob of pass dirs>" [--match mdt::]

Each pass directory holds one ``*_counter_collection.csv``; counters are averaged
per dispatch of each kernel over all passes. Derived columns:
  MFMA%   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)  (rocprofv3's
            MfmaUtil expression; GRBM_GUI_ACTIVE comes summed over the 8 XCDs)
  bf16 TF = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / kernel time (time from the pass's
            own dispatch timestamps; dispatches are serialised under --pmc)
  LDS cf  = SQ_LDS_BANK_CONFLICT cycles per SQ_INSTS_LDS instruction
  HBM GB/s = (FETCH_SIZE + WRITE_SIZE) KB / kernel time
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(k):
    k = k.replace("mdt::", "").replace("void ", "")
    for a in ("(JobPack)", "(IgArgs)", "(WgArgs)", "(ThinConvArgs)", "(ThinTconvArgs)"):
        k = k.replace(a, "")
    return k[:64]


def main():
    root = sys.argv[1]
    match = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--match" else "mdt::"
    val = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for path in sorted(glob.glob(os.path.join(root, "*", "*_counter_collection.csv"))):
        seen = set()
        for r in csv.DictReader(open(path)):
            if match not in r["Kernel_Name"]:
                continue
            k = (r["Kernel_Name"], int(r["Grid_Size"]))  # same template at different layers
            val[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (path, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    mean = lambda xs: sum(xs) / len(xs) if xs else float("nan")
    rows = []
    for k in val:
        c = {n: mean(v) for n, v in val[k].items()}
        t = mean(dur[k])
        grbm = c.get("GRBM_GUI_ACTIVE", float("nan"))
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm / 8 * 1024) * 100 if grbm == grbm else float("nan")
        tf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / t / 1e12 if t > 0 else float("nan")
        lds = c.get("SQ_INSTS_LDS", 0.0)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
        fb = c.get("FETCH_SIZE", 0.0) * 1024
        wb = c.get("WRITE_SIZE", 0.0) * 1024
        bw = (fb + wb) / t / 1e9 if t > 0 else float("nan")
        rows.append((t, k, c, mfma, tf, cf, fb, wb, bw))
    rows.sort(key=lambda r: -r[0])
    print("| kernel | grid | µs (pmc, serial) | waves | MFMA busy % | bf16 TF/s | bf16 GFLOP | LDS instr | LDS conflict cyc/instr | fetch KB | write KB | HBM GB/s |")
    print("|---" * 12 + "|")
    tot_fl = 0.0
    for t, k, c, mfma, tf, cf, fb, wb, bw in rows:
        fl = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
        tot_fl += fl
        print(f"| `{short(k[0])}` | {k[1]} | {t * 1e6:.1f} | {c.get('SQ_WAVES', 0):.0f} | {mfma:.1f} | {tf:.1f} | {fl / 1e9:.3f} | "
              f"{c.get('SQ_INSTS_LDS', 0):.3g} | {cf:.3f} | {fb / 1024:.0f} | {wb / 1024:.0f} | {bw:.0f} |")
    print(f"\nbf16 MFMA work per dispatch set: {tot_fl / 1e9:.3f} GFLOP")


if __name__ == "__main__":
    main()
