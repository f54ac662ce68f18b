#!/bin/bash
# round 4, session 8: in-step A/B of the LDS-DMA piece form (FLAT default vs buffer form in gemm_pp and
# wgrad_pp), interleaved bench runs, then the wgrad ablations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4p}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/flat_$r.log 2>&1 || exit 1
  echo "flat r=$r $(v $O/flat_$r.log)"
  ND_GEMM_PP_VARIANT=1024 ND_WGRAD_VARIANT=b timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/buf_$r.log 2>&1 || exit 1
  echo "buf  r=$r $(v $O/buf_$r.log)"
done
timeout -k 10 300 python -u scripts/wgrad_abl.py --abl 1,2,4,8,16,3,7,31 > $O/abl.log 2>&1
rc=$?; cat $O/abl.log; exit $rc
