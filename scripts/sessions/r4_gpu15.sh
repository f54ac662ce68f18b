#!/bin/bash
# round 4, session 15: full GPU test suite at HEAD, then the per-kernel PMC table of the bf16 bench step
# (three counter passes, kernel-trace only, merged)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4x}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -4 $O/test.log; [ $rc -eq 0 ] || exit $rc
bash scripts/sessions/r3_pmc.sh > $O/pmc.log 2>&1
rc=$?; tail -30 $O/pmc.log; cp gpurun_out/pmc/merged.md $O/pmc_merged.md 2>/dev/null; exit $rc
