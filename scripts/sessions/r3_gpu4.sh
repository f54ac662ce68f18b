#!/bin/bash
# round 3, session 4: ping-pong GEMM numerics (prologue fix), ablation timing, PMC vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --check-only > $O/check.log 2>&1; echo "check exit $?" >> $O/check.log
tail -25 $O/check.log
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --ablate 0,1,2,3,4,8,15 --rounds 5 > $O/ablate.log 2>&1 && tail -5 $O/ablate.log || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o pp -- python3 scripts/gemm_pmc.py --pp --iters 5 > $O/pmc.log 2>&1; echo "pmc rc $?" >> $O/pmc.log
tail -2 $O/pmc.log
