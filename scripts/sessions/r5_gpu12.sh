#!/bin/bash
# round 5 (16 HW queues): flag A/B -- micro-batch 256, unfenced wgrad side stream, own plain GEMMs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['config']['micro_batch'], d['proj_gemm'])"; }
run() { local arm=$1; shift; timeout -k 10 300 python bench.py --steps 8 --warmup 2 "$@" > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }; echo "$arm r=$r $(v $O/${arm}_$r.log)"; }
for r in 1 2; do
  run base
  run mb256 --micro-batch 256
  run unfenced --wgrad-overlap 2
  run pp --proj-gemm pp
  run w128 --proj-gemm w128
done
