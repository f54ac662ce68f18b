#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV (run_kernel_stats.csv) into a markdown table."""
import csv
import sys


def main(path, top=25, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"]
        if name.startswith("void "):
            name = name[5:]
        if name.startswith("(anonymous namespace)::"):
            name = name[len("(anonymous namespace)::"):]
        name = name.split("(")[0][:90]
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.1f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    print(f"\ntotal kernel time: {tot/1e6:.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
