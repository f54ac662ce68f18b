#!/bin/bash
# round 4, session 5: FLAT-global LDS-DMA pieces in the step's own GEMMs (gemm_pp fused kernels, wgrad_pp):
# tail-shape numerics with the flat form, then the interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4m}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u -c "
import sys; sys.path.insert(0, 'scripts')
from nanodiloco_amd import ops; ops.set_backend('hip')
from nanodiloco_amd.ops import gemm as G
import gemm_pp_bench as B
G.set_pp_variant(1024)
sys.exit(1 if B.check() else 0)" > $O/check.log 2>&1 &&
timeout -k 10 300 python -u scripts/gdma_ab.py --rounds 5 > $O/ab.log 2>&1
rc=$?; cat $O/check.log $O/ab.log; exit $rc
