#!/bin/bash
# round 4, session 6: HEAD validation -- the GPU test suite, the bf16 bench, a kernel-trace profile of it,
# and the overlapped outer step on a live one-rank RCCL group (H = 1: every step carries an outer step;
# serialized vs --overlap-outer) for Llama-150M and Llama-1B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4n}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
step() { echo "== $1: $(tail -c 400 $O/$1.log | grep -o '"ms_per_step": [0-9.]*\|"outer_step_ms": [0-9.]*\|"value": [0-9.]*\|"comm_backend": "[a-z]*"' | tr '\n' ' ')"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
step bench
for m in 150m 1b; do
  for ov in "" "--overlap-outer"; do
    n=ov_${m}${ov:+_ov}
    timeout -k 10 400 python bench.py --model llama_$m.json --backend nccl --inner-steps 1 --steps 4 --warmup 2 $ov > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
    step $n
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -30 $O/kernel_stats.md
