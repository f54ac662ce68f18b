#!/bin/bash
# round 3, session 18: ping-pong attention forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd_variants" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
FWD_ONLY=1 VARIANTS=d,d:32,p,p3,pq timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
