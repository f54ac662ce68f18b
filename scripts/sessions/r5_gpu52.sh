#!/bin/bash
# round 5: embedding gathers straight into the bf16 residual stream (no cast pass): tests + fp8 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5az
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fp8_gpu.py -m gpu -k "embedding or residual or deterministic or trajectory or hip_vs_torch" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["residual_dtype"])'; }
timeout -k 10 300 python bench.py --fp8 > $O/f8.log 2>&1 || { tail -5 $O/f8.log; exit 1; }
echo "fp8 $(v $O/f8.log)"
timeout -k 10 300 python bench.py --residual-dtype bf16 > $O/b16.log 2>&1 || { tail -5 $O/b16.log; exit 1; }
echo "bf16-res $(v $O/b16.log)"
timeout -k 10 300 python bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "default $(v $O/b.log)"
