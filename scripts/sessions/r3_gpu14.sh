#!/bin/bash
# round 3, session 14: texture-addresser (TA) pressure of the ping-pong GEMM vs hipBLASLt (q|k|v fwd shape)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -o "\bT[ACD][A-Z_]*\b" $O/counters.txt | sort -u > $O/ta_names.txt || true
wc -l $O/ta_names.txt
TA=$(grep -E "^TA_(TA_BUSY|BUSY)" $O/ta_names.txt | head -1)
TB=$(grep -E "^TA_BUFFER_(READ_)?WAVEFRONTS$|^TA_BUFFER_WAVEFRONTS" $O/ta_names.txt | head -1)
TC=$(grep -E "^TA_ADDR_STALLED_BY_TC_CYCLES|^TA_DATA_STALLED_BY_TC_CYCLES" $O/ta_names.txt | head -1)
TD=$(grep -E "^TD_TD_BUSY|^TD_BUSY" $O/ta_names.txt | head -1)
echo "using: $TA $TB | $TC $TD"
[ -n "$TA" ] || exit 0
timeout -s KILL 90 rocprofv3 --pmc ${TA}_sum ${TB:+${TB}_sum} GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc1 -o p -- python3 scripts/gemm_pmc.py --iters 5 > $O/pmc1.log 2>&1; echo "pmc1 rc $?"
[ -n "$TC" ] && timeout -s KILL 90 rocprofv3 --pmc ${TC}_sum ${TD:+${TD}_sum} GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc2 -o p -- python3 scripts/gemm_pmc.py --iters 5 > $O/pmc2.log 2>&1; echo "pmc2 rc $?"
