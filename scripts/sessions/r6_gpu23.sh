#!/bin/bash
# round 6 session 23: the coefficient form as the default -- the whole GPU suite, smoke, bf16 and --fp8 bench, closing profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_bf16.log 2>&1 || { tail -20 $O/bench_bf16.log; exit 1; }
tail -1 $O/bench_bf16.log | cut -c1-220
timeout -k 10 300 python -u bench.py --fp8 --steps 20 --warmup 5 > $O/bench_fp8.log 2>&1 || { tail -20 $O/bench_fp8.log; exit 1; }
tail -1 $O/bench_fp8.log | cut -c1-220
# closing profiles at this HEAD: serial kernel stats of the bf16 / --fp8 step, PMC table of the bf16 step
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof_bf16.log 2>&1 || { tail -5 $O/prof_bf16.log; exit 1; }
f=$(find $O/prof_bf16 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_bf16.md; head -16 $O/kernel_stats_bf16.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 bench.py --fp8 --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof_fp8.log 2>&1 || { tail -5 $O/prof_fp8.log; exit 1; }
f=$(find $O/prof_fp8 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_fp8.md; head -16 $O/kernel_stats_fp8.md
bash scripts/sessions/r3_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc/merged.md $O/pmc_merged.md && head -24 $O/pmc_merged.md
rm -rf $O/prof_bf16 $O/prof_fp8
