#!/bin/bash
# round 3, session 2: ping-pong GEMM numerics + timing A/B, then the full GPU tests / smoke / bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 240 python -u scripts/gemm_pp_bench.py --rounds 3 > $O/pp.log 2>&1; rc=$?
echo "pp exit $rc" >> $O/pp.log
tail -20 $O/pp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest exit $?" >> $O/pytest.log
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --backend nccl --steps 10 --warmup 3 > $O/bench_nccl.log 2>&1 && tail -1 $O/bench_nccl.log
