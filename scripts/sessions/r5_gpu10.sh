#!/bin/bash
# round 5: one-rank PG cost with claimed compute queues: stream priority of the communicators
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['comm_backend'], d.get('comm_impl'))"; }
run() { local arm=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 6 --warmup 2 $BARGS > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }; echo "$arm r=$r $(v $O/${arm}_$r.log)"; }
for r in 1 2; do
  BARGS="--backend none"; run none X=1
  BARGS=""; run rccl_lowprio ND_COMM_PRIORITY=normal
  BARGS=""; run rccl_q16_lowprio ND_COMM_PRIORITY=normal GPU_MAX_HW_QUEUES=16
  BARGS=""; run rccl_q16 GPU_MAX_HW_QUEUES=16
done
