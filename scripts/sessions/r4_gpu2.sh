#!/bin/bash
# round 4, session 2: w128 ablations (timing only) and two PMC passes: w128 vs hipBLASLt vs ping-pong
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/${SESSION:-r4c}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/w128_probe.py ablate --abl ${ABL:-1,2,4,8,16,31} > $O/ablate.log 2>&1
rc=$?; cat $O/ablate.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/pmc1 -o p1 -- python3 $R/scripts/w128_probe.py pmc > $R/$O/pmc1.log 2>&1
rc=$?; tail -2 $R/$O/pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/pmc2 -o p2 -- python3 $R/scripts/w128_probe.py pmc > $R/$O/pmc2.log 2>&1
rc=$?; tail -2 $R/$O/pmc2.log; [ $rc -eq 0 ] || exit $rc
cd $R
for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== $f"; python3 scripts/pmc_summary.py $f; done
