#!/bin/bash
# round 5: q|k|v epilogue -- v waves take the plain store body (no table loads), q/k waves rotate without selects
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ALT=nanodiloco_amd/_lib/alt/libnd_kernels_131533a.so
timeout -k 10 200 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_gemm_pp_f8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_kernels.py --alt $ALT --what epi --rounds 5 > $O/epi.log 2>&1 || { tail -5 $O/epi.log; exit 1; }
grep "speedup" $O/epi.log
timeout -k 10 300 python scripts/ab_kernels.py --alt $ALT --what step --rounds 4 --iters 3 > $O/step.log 2>&1 || { tail -5 $O/step.log; exit 1; }
grep "speedup" $O/step.log
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/fp8test.log 2>&1; rc=$?; tail -3 $O/fp8test.log; [ $rc -eq 0 ] || exit $rc
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['final_loss'])"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --fp8 --steps 8 --warmup 2 > $O/f8lm_$r.log 2>&1 || { tail -3 $O/f8lm_$r.log; exit 1; }
  echo "fp8 lm-head fp8  r=$r $(v $O/f8lm_$r.log)"
  timeout -k 10 300 python bench.py --fp8 --fp8-lm-head 0 --steps 8 --warmup 2 > $O/f8bf_$r.log 2>&1 || { tail -3 $O/f8bf_$r.log; exit 1; }
  echo "fp8 lm-head bf16 r=$r $(v $O/f8bf_$r.log)"
done
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/bf16.log 2>&1 || { tail -3 $O/bf16.log; exit 1; }
echo "bf16 $(v $O/bf16.log)"
