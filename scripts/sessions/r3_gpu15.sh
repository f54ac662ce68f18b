#!/bin/bash
# round 3, session 15: pipelined attention forward -- numerics + A/B vs the round-2 kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python3 scripts/attn_pmc.py > $O/pmc.log 2>&1; echo "pmc rc $?"
f=$(find $O/pmc -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 scripts/pmc_summary.py $f > $O/pmc_summary.md; cat $O/pmc_summary.md
