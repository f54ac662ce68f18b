#!/bin/bash
# round 3, session 20: attention tests after removing the rejected kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3t
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
VARIANTS=d,d:32,d:128,d:160 BWD_VARIANTS=o,o4 timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
