#!/bin/bash
# One GPU session: kernel/model tests, then a short bench. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${SKIP_BENCH:-}" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
echo "bench rc=$brc"
exit $brc
