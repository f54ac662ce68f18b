#!/bin/bash
# in-step A/B with the weight-gradient side stream on (default): plain products on hipBLASLt (fenced side stream)
# vs the own ping-pong kernel (--proj-gemm pp: no library GEMM to fence except the lm head), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4an
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['proj_gemm'], d.get('wgrad_overlap'))"; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/blas_$r.log 2>&1 || { tail -3 $O/blas_$r.log; exit 1; }
  echo "blas r=$r $(v $O/blas_$r.log)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --proj-gemm pp > $O/pp_$r.log 2>&1 || { tail -3 $O/pp_$r.log; exit 1; }
  echo "pp   r=$r $(v $O/pp_$r.log)"
done
