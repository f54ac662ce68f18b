#!/bin/bash
# staggered-DMA wgrad variant: correctness + in-process A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2w
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r2w/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r2w/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/wgrad_env_ab.py --variants ,stg --rounds 7 > gpurun_out/r2w/ab.log 2>&1 || exit $?
cat gpurun_out/r2w/ab.log
