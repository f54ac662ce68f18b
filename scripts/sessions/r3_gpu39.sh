#!/bin/bash
# round 3, session 39: attention output stores as 16-B chunks (permlane32 pairing) vs HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3am
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_*.so --what attnk --rounds 9 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
