#!/bin/bash
# round 4, session 10: fp8 step on the own fp8 ping-pong GEMM with fused epilogues -- model-level tests,
# then interleaved bench A/B: bf16 | --fp8 (pp + fused, default) | --fp8 pp unfused | --fp8 hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4r}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -5 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/bf16_$r.log 2>&1 || { tail -3 $O/bf16_$r.log; exit 1; }
  echo "bf16 r=$r $(v $O/bf16_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 > $O/f8pp_$r.log 2>&1 || { tail -3 $O/f8pp_$r.log; exit 1; }
  echo "fp8 pp fused r=$r $(v $O/f8pp_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --fp8-fused-epi 0 > $O/f8ppu_$r.log 2>&1 || { tail -3 $O/f8ppu_$r.log; exit 1; }
  echo "fp8 pp unfused r=$r $(v $O/f8ppu_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --fp8-gemm hipblaslt > $O/f8bl_$r.log 2>&1 || { tail -3 $O/f8bl_$r.log; exit 1; }
  echo "fp8 hipblaslt r=$r $(v $O/f8bl_$r.log)"
done
