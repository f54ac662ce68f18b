#!/bin/bash
# round 5: checkpoint staging / resume auto on the GPU (multi-rank GPU tests incl. checkpoints) + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5aq
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multirank_gpu.py tests/test_rccl_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
