#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q -s --timeout 200 --timeout-method thread -k "one_step or side_stream" > $O/t.log 2>&1; rc=$?; grep "bf16\|passed\|failed\|Error" $O/t.log | head -40; exit $rc
