#!/bin/bash
# round 5: bf16 residual stream (--residual-dtype bf16): kernel / model tests, then an interleaved bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ax
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py -m gpu -k "rmsnorm or residual or trajectory or hip_vs_torch or quant" > $O/test.log 2>&1
rc=$?; tail -4 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["residual_dtype"])'; }
for rd in 1 2 3; do
  for r in fp32 bf16; do
    timeout -k 10 300 python bench.py --residual-dtype $r > $O/b_${r}_$rd.log 2>&1 || { tail -5 $O/b_${r}_$rd.log; exit 1; }
    echo "r$rd $(v $O/b_${r}_$rd.log)"
  done
done
