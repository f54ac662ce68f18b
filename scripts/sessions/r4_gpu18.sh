#!/bin/bash
# round 4, session 18: fp8 side outputs packed once (rmsnorm / swiglu), rmsnorm bwd at 4 waves per SIMD --
# fp8 tests, then the fp8 bench and its kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4aa}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/bf16.log 2>&1 || exit 1
echo "bf16 $(v $O/bf16.log)"
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 > $O/f8.log 2>&1 || exit 1
echo "fp8 $(v $O/f8.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --fp8 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; grep -i "rmsnorm\|swiglu\|total" $O/kernel_stats.md
