#!/bin/bash
# round 3, session 46 (final): HEAD validation: full GPU suite, smoke, bench (bf16 / fp8 / 1B), kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3at
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/pytest.log
tail -4 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-200 || exit 1
timeout -k 10 300 python bench.py --fp8 > $O/bench_fp8.log 2>&1 && tail -1 $O/bench_fp8.log | cut -c1-200 || exit 1
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 > $O/bench_1b.log 2>&1 && tail -1 $O/bench_1b.log | cut -c1-200 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/rocprof.log 2>&1; echo "rocprof rc $?"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -24 $O/kernel_stats.md
