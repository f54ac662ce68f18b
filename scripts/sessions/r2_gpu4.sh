#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcg4
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --rounds 3 --variants ${VARIANTS:-4:0,4:2,4:4,4:8} > gpurun_out/gemm_ab3.log 2>&1 || exit $?
cat gpurun_out/gemm_ab3.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for g in 4; do
P="python3 scripts/gemm_pmc.py --iters 3 --variants 5"
ND_GEMM_GROUP_M=$g timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcg4 -o sq$g -- $P > gpurun_out/pmcg4/sq$g.log 2>&1 || exit $?
ND_GEMM_GROUP_M=$g timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcg4 -o tc$g -- $P > gpurun_out/pmcg4/tc$g.log 2>&1 || exit $?
python3 scripts/pmc_dump.py $(find gpurun_out/pmcg4 -name "*$g""_counter_collection.csv") > gpurun_out/pmcg4/summary$g.txt 2>&1
grep -A30 "gemm4\|Cijk" gpurun_out/pmcg4/summary$g.txt
done
