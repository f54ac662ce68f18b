#!/bin/bash
# round 5 baseline: bf16 bench (blas / pp plain products, interleaved) and the ten plain products in isolation
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/blas_$r.log 2>&1 || { tail -3 $O/blas_$r.log; exit 1; }
  echo "blas r=$r $(v $O/blas_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --proj-gemm pp > $O/pp_$r.log 2>&1 || { tail -3 $O/pp_$r.log; exit 1; }
  echo "pp   r=$r $(v $O/pp_$r.log)"
done
timeout -k 10 400 python scripts/gemm_pp_bench.py --tokens 131072 --rounds 3 > $O/gemm.log 2>&1 || { tail -5 $O/gemm.log; exit 1; }
tail -30 $O/gemm.log
