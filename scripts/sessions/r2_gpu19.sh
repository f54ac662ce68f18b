#!/bin/bash
# new trajectory + bench-shape attention tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2t
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -k "trajectory or flash_attention_fwd_bwd" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r2t/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r2t/pytest.log | cut -c1-250 | tail -20
exit $rc
