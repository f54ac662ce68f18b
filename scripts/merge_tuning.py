#!/usr/bin/env python3
"""Merge a freshly tuned TunableOp CSV (scripts/tune_gemms.py, OUT=...) into the shipped table
nanodiloco_amd/tuning/tunableop_gfx950.csv.

The validator lines (torch / HIP / hipBLASLt / rocBLAS versions, arch) of both files must agree --
a table tuned on another software stack is refused.  Result lines of the new file replace lines of
the shipped table with the same (op, shape signature); all others are kept.

    python scripts/merge_tuning.py gpurun_out/tune_new.csv [--dry-run]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops.tuned_gemm import DEFAULT_FILE  # noqa: E402


def read(path):
    validators, results = {}, {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                validators[parts[1]] = ",".join(parts[2:])
            else:
                results[(parts[0], parts[1])] = line
    return validators, results


def main():
    new_path = sys.argv[1]
    dry = "--dry-run" in sys.argv
    v_old, r_old = read(DEFAULT_FILE)
    v_new, r_new = read(new_path)
    diff = {k: (v_old.get(k), v_new.get(k)) for k in set(v_old) | set(v_new) if v_old.get(k) != v_new.get(k)}
    if diff:
        raise SystemExit(f"validator mismatch, refusing to merge: {diff}")
    added = [k for k in r_new if k not in r_old]
    changed = [k for k in r_new if k in r_old and r_old[k] != r_new[k]]
    merged = dict(r_old)
    merged.update(r_new)
    print(f"{len(r_old)} shipped + {len(added)} new, {len(changed)} re-tuned -> {len(merged)} entries")
    for k in added:
        print("  new:", r_new[k])
    if dry:
        return
    with open(DEFAULT_FILE, "w") as f:
        for k, v in v_old.items():
            f.write(f"Validator,{k},{v}\n")
        for k in sorted(merged):
            f.write(merged[k] + "\n")
    print("wrote", DEFAULT_FILE)


if __name__ == "__main__":
    main()
