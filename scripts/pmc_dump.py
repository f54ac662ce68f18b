#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc CSVs (one or more passes).

    python scripts/pmc_dump.py gpurun_out/pmc/*counter_collection.csv
"""
import collections
import csv
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60]
        key = (name, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for key, ctrs in per.items():
        for c, v in ctrs.items():
            rows[key[0]][c].append(v)
        rows[key[0]]["us"].append(dur[key])
for name, ctrs in rows.items():
    avg = {c: sum(v) / len(v) for c, v in ctrs.items()}
    print(f"== {name}  (n={len(ctrs['us'])})")
    wc = avg.get("SQ_WAVE_CYCLES")
    for c in sorted(avg):
        extra = ""
        if wc and c.startswith("SQ_WAIT") or (wc and c.startswith("SQ_ACTIVE")):
            extra = f"  ({avg[c] / wc:.3f} of wave cycles)"
        if c == "SQ_VALU_MFMA_BUSY_CYCLES" and "GRBM_GUI_ACTIVE" in avg:
            extra = f"  (MFMA busy {100 * avg[c] / avg['GRBM_GUI_ACTIVE'] / 128:.1f} %)"
        print(f"   {c:32s} {avg[c]:16.1f}{extra}")
