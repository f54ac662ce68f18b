#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection CSV per kernel.

Default counter set (scripts/pmc_session.sh): ratios vs SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE.
Any other counter set: per-call averages of every collected counter.
"""
import collections
import csv
import sys

DEFAULT = {"SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
           "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES"}


def main(path, top=12):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    calls = collections.defaultdict(set)
    seen = set()
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:48]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r["Dispatch_Id"], r["Process_Id"])
        calls[name].add(key)
        if key not in seen:
            seen.add(key)
            dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ctrs = sorted({c for d in agg.values() for c in d})
    order = sorted(agg, key=lambda k: -dur[k])[:top]
    if not DEFAULT <= set(ctrs):
        print("| kernel | calls | avg us | " + " | ".join(ctrs) + " |")
        print("|---" * (3 + len(ctrs)) + "|")
        for name in order:
            k = max(1, len(calls[name]))
            print(f"| `{name}` | {k} | {dur[name] / k:.1f} | " + " | ".join(f"{agg[name][c] / k:.4g}" for c in ctrs) + " |")
        return
    print("| kernel | calls | avg us | WAIT_ANY | WAIT_INST | VALU | LDS | MFMA_BUSY/GUI | LDS_BANK_CONFL/LDS |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name in order:
        d = agg[name]
        k = max(1, len(calls[name]))
        wc = max(1.0, d["SQ_WAVE_CYCLES"])
        gui = max(1.0, d.get("GRBM_GUI_ACTIVE", 1.0))
        print(f"| `{name}` | {k} | {dur[name] / k:.1f} | {d['SQ_WAIT_ANY'] / wc:.2f} | "
              f"{d['SQ_WAIT_INST_ANY'] / wc:.2f} | {d['SQ_ACTIVE_INST_VALU'] / wc:.2f} | {d['SQ_ACTIVE_INST_LDS'] / wc:.2f} | "
              f"{d['SQ_VALU_MFMA_BUSY_CYCLES'] / gui:.2f} | {d['SQ_LDS_BANK_CONFLICT'] / max(1, d['SQ_ACTIVE_INST_LDS']):.3f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
