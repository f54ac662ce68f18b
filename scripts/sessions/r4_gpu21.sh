#!/bin/bash
# round 4, session 21: fp8 weight gradients on the side stream too -- fp8 tests, then --fp8 with the overlap
# on / off, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4ae}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fp8 --wgrad-overlap 0 > $O/f8_$r.log 2>&1 || exit 1
  echo "fp8 overlap 0 r=$r $(v $O/f8_$r.log)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fp8 > $O/f8wo_$r.log 2>&1 || exit 1
  echo "fp8 overlap 1 r=$r $(v $O/f8wo_$r.log)"
done
