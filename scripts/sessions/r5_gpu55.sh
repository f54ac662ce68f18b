#!/bin/bash
# round 5: the CE kernel writes the fp8 lm head's e5m2 dlogits directly: tests + fp8 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bc
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -m gpu > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["residual_dtype"])'; }
for rd in 1 2; do
  timeout -k 10 300 python bench.py --fp8 > $O/f8_$rd.log 2>&1 || { tail -5 $O/f8_$rd.log; exit 1; }
  echo "fp8 r$rd $(v $O/f8_$rd.log)"
done
timeout -k 10 300 python bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "bf16 $(v $O/b.log)"
