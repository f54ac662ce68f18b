#!/bin/bash
# round 5: GPU fault drill (one-rank RCCL job: crash, torchrun restart, resume auto)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ar
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_multirank_gpu.py -k crash > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
