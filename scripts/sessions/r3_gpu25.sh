#!/bin/bash
# round 3, session 25: dQ tile loop unrolled by buffer parity: 3 waves/SIMD (9 spills, working tree) vs 2 waves (alt) vs pre-unroll (alt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
for alt in nanodiloco_amd/_lib/alt/libnd_kernels_3d6e45d.so nanodiloco_amd/_lib/alt/libnd_kernels_*_dq2.so; do
  echo "alt = $alt"
  timeout -k 10 200 python -u scripts/ab_kernels.py --alt $alt --what attnk --rounds 7 > $O/ab.log 2>&1 || exit 1
  cat $O/ab.log
done
