#!/bin/bash
# round 3, session 1: full GPU tests (incl. the new RCCL one-rank tests), smoke, default bench,
# bench under torchrun with a live one-rank RCCL communicator
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest exit $?" >> $O/pytest.log
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --backend nccl --steps 10 --warmup 3 > $O/bench_nccl.log 2>&1 && tail -1 $O/bench_nccl.log
