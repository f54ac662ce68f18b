#!/bin/bash
# round 5: weight-gradient s_setprio variants (p1 static priority for the younger group, p2 none) vs default; grouped MLP launch on for all arms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bj
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2 3; do
  for v in "" p1 p2; do
    ND_WGRAD_VARIANT=$v timeout -k 10 120 python scripts/wgrad_variant_time.py >> $O/kern.log 2>&1 || { tail -5 $O/kern.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kern.log
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2 3; do
  for v in "" p1 p2; do
    ND_WGRAD_VARIANT=$v timeout -k 10 300 python bench.py > $O/b_${v:-d}_$rd.log 2>&1 || { tail -5 $O/b_${v:-d}_$rd.log; exit 1; }
    echo "bench ${v:-default} r$rd $(b $O/b_${v:-d}_$rd.log)"
  done
done
