#!/bin/bash
# round 5 final: full GPU suite + smoke + bench at the closing HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bh
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -5 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-300
