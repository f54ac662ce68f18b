#!/usr/bin/env python3
"""Check that a TunableOp table takes effect: time the plain projection GEMMs (torch.mm, the bench's
layouts) with the table loaded vs TunableOp off.  Usage: python scripts/tuned_check.py TABLE.csv [tokens]"""
import os
import sys

import torch
import torch.cuda.tunable as tunable


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    path = sys.argv[1]
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    shapes = {"o fwd": (1024, 1024), "down fwd": (1024, 2688), "qkv dgrad": (1024, 3072), "gu dgrad": (1024, 5376)}
    ops = {}
    for k, (n, kk) in shapes.items():
        a, b = r(M, kk), r(n, kk)
        out = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        ops[k] = (a, b, out)
    res = {}
    for rd in range(3):
        for mode in ("off", "table"):
            tunable.enable(mode == "table")
            if mode == "table":
                tunable.tuning_enable(False)
                tunable.record_untuned_enable(False)
                tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tc_{os.getpid()}.csv"))
                if rd == 0:
                    print("read_file:", tunable.read_file(path), "results:", len(tunable.get_results()), flush=True)
                    print([x for x in tunable.get_results() if "131072" in str(x)], flush=True)
            for k, (a, b, out) in ops.items():
                res.setdefault((k, mode), []).append(timed(lambda: torch.mm(a, b.t(), out=out)))
                res.setdefault((k, mode + "-noout"), []).append(timed(lambda: torch.mm(a, b.t())))
    for k in shapes:
        print(f"{k:10s} " + " | ".join(f"{m} {sorted(res[(k, m)])[1]:7.1f} us" for m in ("off", "table", "off-noout", "table-noout")), flush=True)


if __name__ == "__main__":
    main()
