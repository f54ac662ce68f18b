#!/bin/bash
# PMC counter run (kernel-trace + counters only; never combined with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"}
timeout -k 10 ${T:-600} rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/pmc -o ${NAME:-run} -- python3 ${PROG:-bench.py} ${ARGS:---steps 1 --warmup 1} > gpurun_out/pmc/${NAME:-run}.log 2>&1
rc=$?
tail -3 gpurun_out/pmc/${NAME:-run}.log
echo "pmc rc=$rc"
exit $rc
