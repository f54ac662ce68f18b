#!/usr/bin/env python3
"""Merge several rocprofv3 --pmc passes (one counter set each; the hardware cannot collect them in
one pass) into one per-kernel table: MFMA-pipe utilisation, stall ratios, HBM bytes and the achieved
HBM bandwidth.

    python scripts/pmc_merge.py gpurun_out/pmc/sq_counter_collection.csv \\
        gpurun_out/pmc/fetch_counter_collection.csv gpurun_out/pmc/write_counter_collection.csv

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KB (TCC traffic to/from memory).
SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE is summed over the 32 CUs x 4 SIMDs of an XCD's
counters, so 128 = every MFMA pipe busy; the table reports it as a percentage of 128.
"""
import collections
import csv
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    calls = collections.defaultdict(set)
    seen = set()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:44]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r["Dispatch_Id"], r["Process_Id"])
        calls[name].add(key)
        if key not in seen:
            seen.add(key)
            dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return agg, dur, calls


def main(paths, top=16):
    agg = collections.defaultdict(dict)
    dur, ncall = {}, {}
    for p in paths:
        a, d, c = load(p)
        for k in a:
            n = max(1, len(c[k]))
            for ctr, v in a[k].items():
                agg[k][ctr] = v / n
            # per-pass duration of the same kernels: keep the first pass's (counters perturb timing
            # little; each pass times its own dispatches)
            dur.setdefault(k, d[k] / n)
            ncall.setdefault(k, n)
    order = sorted(dur, key=lambda k: -dur[k] * ncall[k])[:top]
    print("| kernel | calls | avg us | MFMA busy % | WAIT_ANY | WAIT_INST | HBM read GB | HBM write GB | HBM TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in order:
        d = agg[k]
        us = dur[k]
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        gui = d.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = f"{100 * d['SQ_VALU_MFMA_BUSY_CYCLES'] / gui / 128:.1f}" if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in d else "-"
        wa = f"{d['SQ_WAIT_ANY'] / wc:.2f}" if wc and "SQ_WAIT_ANY" in d else "-"
        wi = f"{d['SQ_WAIT_INST_ANY'] / wc:.2f}" if wc and "SQ_WAIT_INST_ANY" in d else "-"
        rd = d.get("FETCH_SIZE")
        wr = d.get("WRITE_SIZE")
        rd_gb = f"{rd / 1e6:.3f}" if rd is not None else "-"
        wr_gb = f"{wr / 1e6:.3f}" if wr is not None else "-"
        bw = "-"
        if rd is not None and wr is not None and us > 0:
            bw = f"{(rd + wr) * 1e3 / (us * 1e-6) / 1e12:.2f}"
        print(f"| `{k}` | {ncall[k]} | {us:.1f} | {mfma} | {wa} | {wi} | {rd_gb} | {wr_gb} | {bw} |")


if __name__ == "__main__":
    main(sys.argv[1:])
