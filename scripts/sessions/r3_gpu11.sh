#!/bin/bash
# round 3, session 11: HEAD validation (ping-pong GEMM tests incl. the model-level fused test), default
# bench, fp8 bench, and a rocprofv3 kernel profile of the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/pytest.log
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-200 || exit 1
timeout -k 10 300 python bench.py --fp8 > $O/bench_fp8.log 2>&1 && tail -1 $O/bench_fp8.log | cut -c1-200 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $O/rocprof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 32 > $O/kernel_stats.md
head -24 $O/kernel_stats.md
