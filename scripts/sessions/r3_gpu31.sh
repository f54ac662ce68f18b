#!/bin/bash
# round 3, session 31: attention (ILP-variant default) + model GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or flash or model or trajectory" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
