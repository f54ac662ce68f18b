#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection CSV per kernel (ratios vs SQ_WAVE_CYCLES)."""
import collections
import csv
import sys


def main(path, top=12):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    n = collections.Counter()
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVE_CYCLES":
            n[name] += 1
            dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("| kernel | calls | avg us | WAIT_ANY | WAIT_INST | VALU | LDS | MFMA_BUSY/GUI | LDS_BANK_CONFL/LDS |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, d in sorted(agg.items(), key=lambda kv: -dur[kv[0]])[:top]:
        wc = max(1.0, d["SQ_WAVE_CYCLES"])
        gui = max(1.0, d.get("GRBM_GUI_ACTIVE", 1.0))
        print(f"| `{name}` | {n[name]} | {dur[name] / max(1, n[name]):.1f} | {d['SQ_WAIT_ANY'] / wc:.2f} | "
              f"{d['SQ_WAIT_INST_ANY'] / wc:.2f} | {d['SQ_ACTIVE_INST_VALU'] / wc:.2f} | {d['SQ_ACTIVE_INST_LDS'] / wc:.2f} | "
              f"{d['SQ_VALU_MFMA_BUSY_CYCLES'] / gui:.2f} | {d['SQ_LDS_BANK_CONFLICT'] / max(1, d['SQ_ACTIVE_INST_LDS']):.3f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
