#!/bin/bash
# round 5: long-context attention tests (T = 4096 / 8192) vs the fp32 reference
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5be
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "flash_attention_fwd_bwd" > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; exit $rc
