#!/bin/bash
# round 3, session 42: --fp8 with some projections kept on the bf16 fused-epilogue GEMMs (A/B, interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ap
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py > $O/pytest_fp8.log 2>&1; rc=$?; tail -3 $O/pytest_fp8.log; echo "fp8 tests rc $rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in none rope mlp both; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --fp8 --fp8-keep-fused $k > $O/bench_${k}_$r.log 2>&1 || exit 1
    echo "$k $r $(tail -1 $O/bench_${k}_$r.log | cut -c90-150)"
  done
done
