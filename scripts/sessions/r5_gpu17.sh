#!/bin/bash
# round 5: grouped MLP weight gradients (nd_wgrad2) -- tests, then an interleaved bench A/B (--wgrad-group 0/1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rd in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --wgrad-group $g > $O/b_${g}_$rd.log 2>&1 || { tail -5 $O/b_${g}_$rd.log; exit 1; }
    echo "group=$g round=$rd $(tail -1 $O/b_${g}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
