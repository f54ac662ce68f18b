#!/bin/bash
# round 4, session 11: ds_read_b64_tr_b8 semantics probe, then the fp8 weight-gradient kernel: numerics and
# timing vs the bf16 one (plus the fp8 projection GEMMs again)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4s}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_probe_gpu.py -x -q -s --timeout 120 --timeout-method thread > $O/probe.log 2>&1
rc=$?; tail -5 $O/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gemm_pp_f8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -15 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_pp_f8_bench.py --rounds 5 > $O/bench.log 2>&1
rc=$?; cat $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/fp8test.log 2>&1
rc=$?; tail -5 $O/fp8test.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/bf16_$r.log 2>&1 || { tail -3 $O/bf16_$r.log; exit 1; }
  echo "bf16 r=$r $(v $O/bf16_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 > $O/f8_$r.log 2>&1 || { tail -3 $O/f8_$r.log; exit 1; }
  echo "fp8 (wgrad bf16) r=$r $(v $O/f8_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --fp8-wgrad > $O/f8w_$r.log 2>&1 || { tail -3 $O/f8w_$r.log; exit 1; }
  echo "fp8 + fp8 wgrad r=$r $(v $O/f8w_$r.log)"
done
