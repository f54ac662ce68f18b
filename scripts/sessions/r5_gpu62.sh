#!/bin/bash
# round 5: wgrad / model tests after reverting the s_setprio variants (library rebuilt from HEAD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bk
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -k "wgrad or trajectory or smoke" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; exit $rc
