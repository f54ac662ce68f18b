#!/bin/bash
# round 5: PP_DSWIGLU epilogue loads issued before the fat phase's LDS-DMA (variant 2048 = old order): tests + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py tests/test_gemm_pp_f8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rd in 1 2 3; do
  for v in 2048 0; do
    ND_GEMM_PP_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $O/b_${v}_$rd.log 2>&1 || { tail -5 $O/b_${v}_$rd.log; exit 1; }
    echo "bf16 var=$v r$rd $(tail -1 $O/b_${v}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for rd in 1 2; do
  for v in 2048 0; do
    ND_GEMM_PP_VARIANT=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --fp8 > $O/f_${v}_$rd.log 2>&1 || { tail -5 $O/f_${v}_$rd.log; exit 1; }
    echo "fp8 var=$v r$rd $(tail -1 $O/f_${v}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
