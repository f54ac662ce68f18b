#!/bin/bash
# round 3, session 17: 256-query (8-wave) attention forward / dQ blocks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd_variants or dq_variants" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
BWD_VARIANTS=o,o8,k8 VARIANTS=d,d8,d:32,d8:32,d:1,d8:1,d:3,d8:3,d:28,d8:28,d8:4 timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/abl.log 2>&1; rc=$?; cat $O/abl.log; exit $rc
