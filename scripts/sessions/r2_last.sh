#!/bin/bash
# last check at HEAD: full GPU suite, smoke(), default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/last
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/last/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/last/pytest_gpu.log | cut -c1-200 | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/last/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/last/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/last/bench.log 2>&1 || exit $?
tail -1 gpurun_out/last/bench.log | cut -c1-220
