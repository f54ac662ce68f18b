#!/bin/bash
# PMC passes over the own GEMM variants and hipBLASLt on one projection shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcg
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python3 scripts/gemm_pmc.py --iters 3 --variants ${VARIANTS:-1,2}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcg -o sq -- $P > gpurun_out/pmcg/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcg -o p2 -- $P > gpurun_out/pmcg/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcg -o p3 -- $P > gpurun_out/pmcg/p3.log 2>&1; echo "p3 rc=$?"
python3 scripts/pmc_dump.py $(find gpurun_out/pmcg -name "*counter_collection.csv") > gpurun_out/pmcg/summary.txt 2>&1
cat gpurun_out/pmcg/summary.txt
