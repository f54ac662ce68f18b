#!/bin/bash
# round 3, session 10: tile-group sweep of the ping-pong GEMM + end-to-end A/B of the GEMM choice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pp.log 2>&1; echo "pytest exit $?" >> $O/pytest_pp.log
tail -2 $O/pytest_pp.log
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --gms 2,4,8,16 --rounds 5 > $O/gm.log 2>&1 && tail -4 $O/gm.log
for r in 1 2 3; do
for cfg in "blas 0 0" "pp 1 1" "blas 1 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 6 --warmup 2 --proj-gemm $1 --fused-rope $2 --fused-mlp $3 > $O/b.log 2>&1 || { echo "bench failed $cfg"; tail -5 $O/b.log; exit 1; }
  echo "$cfg $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
done
