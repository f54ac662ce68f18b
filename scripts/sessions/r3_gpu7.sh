#!/bin/bash
# round 3, session 7: end-to-end A/B of the projection GEMM choice and the fused epilogues
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pp.log 2>&1; echo "pytest exit $?" >> $O/pytest_pp.log
tail -3 $O/pytest_pp.log
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --ablate 0,8,128 --rounds 5 > $O/abl.log 2>&1 && tail -4 $O/abl.log
for r in 1 2; do
for cfg in "blas 0 0" "pp 1 1" "blas 1 1" "pp 0 0" "blas 1 0" "blas 0 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 6 --warmup 2 --proj-gemm $1 --fused-rope $2 --fused-mlp $3 > $O/b.log 2>&1 || { echo "bench failed $cfg"; tail -5 $O/b.log; exit 1; }
  echo "$cfg $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
done
