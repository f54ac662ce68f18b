#!/bin/bash
# round 5: what does a one-rank process group cost the bench step? (no PG / c10d RCCL only / + own RCCL comm / HW queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['comm_backend'], d.get('comm_impl'))"; }
for r in 1 2; do
  for arm in none c10d rccl q8; do
    case $arm in
      none) args="--backend none";;
      c10d) args="--comm-impl c10d";;
      rccl) args="";;
      q8) args="";;
    esac
    if [ $arm = q8 ]; then
      GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --steps 6 --warmup 2 $args > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }
    else
      timeout -k 10 300 python bench.py --steps 6 --warmup 2 $args > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }
    fi
    echo "$arm r=$r $(v $O/${arm}_$r.log)"
  done
done
