#!/bin/bash
# round 5: fp8 suite incl. the in-op fused-dlogits equivalence test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bg
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -m gpu > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; exit $rc
