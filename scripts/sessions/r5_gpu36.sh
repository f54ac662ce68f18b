#!/bin/bash
# round 5: the o projection's weight gradient deferred and grouped with q|k|v (nd_wgrad2, 64 tiles x 4 splits):
# model tests, then interleaved bench A/B (--wgrad-defer 0/1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5aj
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_inner_ddp_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rd in 1 2 3; do
  for d in 0 1; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --wgrad-defer $d > $O/b_${d}_$rd.log 2>&1 || { tail -5 $O/b_${d}_$rd.log; exit 1; }
    echo "defer=$d r$rd $(tail -1 $O/b_${d}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["wgrad_defer"])')"
  done
done
