#!/bin/bash
# round 3, session 28: plain projection GEMMs on the own ping-pong kernel vs hipBLASLt, interleaved bench A/B + kernel stats of the pp default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for g in blas pp; do
    timeout -k 10 300 python bench.py --proj-gemm $g > $O/bench_${g}_$r.log 2>&1 || exit 1
    echo "$g round $r: $(tail -1 $O/bench_${g}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --proj-gemm pp > $O/rocprof.log 2>&1; echo "rocprof rc $?"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -16 $O/kernel_stats.md
