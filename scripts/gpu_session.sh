#!/bin/bash
# Tests, benches (ours hip / ours torch-ops / reference-equivalent HF eager) and a rocprofv3 kernel
# profile on one GPU box.  Every GPU step has its own time limit; the script stops at the first
# crash or timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
step() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -${TAILN:-4} gpurun_out/$name.log; echo "== $name rc=$rc"; return $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 300 --timeout-method thread; rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
step bench_hip 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} || exit $?
if [ -n "$BENCH2_ARGS" ]; then step bench_hip2 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH2_ARGS} || exit $?; fi
if [ -n "$TORCH_BENCH" ]; then step bench_torchops 600 python bench.py --steps 3 --warmup 1 --ops torch ${BENCH_ARGS} || exit $?; fi
if [ -n "$REF_BENCH" ]; then step ref_baseline 900 python scripts/ref_baseline.py --steps 2 --warmup 1 --micro-batch ${REF_MB:-8} || exit $?; fi
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  step rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ${BENCH_ARGS} || exit $?
fi
exit 0
