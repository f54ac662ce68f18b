#!/bin/bash
# round 5: after removing the superseded wgrad kernels (register-staged 256, 4-wave AGPR): wgrad / model tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ah
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_gemm_pp_f8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
