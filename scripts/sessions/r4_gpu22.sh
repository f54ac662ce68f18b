#!/bin/bash
# round 4, session 22: weight-gradient overlap without fences -- hipBLASLt unfenced (mode 2) and the own
# plain GEMMs (no library GEMM, so no fence), vs the default (hipBLASLt, fenced)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4af}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/d_$r.log 2>&1 || exit 1
  echo "default (blas, fenced) r=$r $(v $O/d_$r.log)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --wgrad-overlap 2 > $O/u_$r.log 2>&1 || exit 1
  echo "blas unfenced r=$r $(v $O/u_$r.log)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --proj-gemm pp > $O/p_$r.log 2>&1 || exit 1
  echo "pp (no fences) r=$r $(v $O/p_$r.log)"
done
