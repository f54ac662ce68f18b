#!/bin/bash
# round 5: GPU_MAX_HW_QUEUES raised by the package + claimed compute queues: one-rank RCCL group vs none
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['comm_backend'], d.get('comm_impl'), d['outer_phase_ms'])"; }
for r in 1 2 3; do
  for arm in none rccl; do
    args=""; [ $arm = none ] && args="--backend none"
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 $args > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }
    echo "$arm r=$r $(v $O/${arm}_$r.log)"
  done
done
