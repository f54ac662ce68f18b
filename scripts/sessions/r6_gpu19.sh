#!/bin/bash
# round 6 session 19: dK/dV query walk and grid order (ND_ATTN_DKDV_ORDER bit 0 = a head's key blocks on one XCD,
# bit 1 = descending query-tile walk): attention fp32-reference tests under orders 2 and 3, then in-process A/B of the
# raw attention (fwd + fused bwd) against side builds with the order default 1 / 2 / 3, and the step for 2 / 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for o in 2 3; do
  ND_ATTN_DKDV_ORDER=$o timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/attn_tests_o$o.log 2>&1 || { tail -30 $O/attn_tests_o$o.log; exit 1; }
  echo "order $o: $(tail -1 $O/attn_tests_o$o.log)"
done
for o in 1 2 3; do
  L=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_o$o.so | head -1)
  timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what attn --rounds 7 --iters 10 > $O/ab_attn_o$o.log 2>&1 || { tail -20 $O/ab_attn_o$o.log; exit 1; }
  echo "== alt order $o (speedup = alt / product time)"; grep speedup $O/ab_attn_o$o.log
done
for o in 2 3; do
  L=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_o$o.so | head -1)
  timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what step --rounds 5 --iters 3 > $O/ab_step_o$o.log 2>&1 || { tail -20 $O/ab_step_o$o.log; exit 1; }
  echo "== step, alt order $o"; grep speedup $O/ab_step_o$o.log
done
