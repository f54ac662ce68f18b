#!/bin/bash
# Round-3 PMC profile of the Llama-150M bf16 bench step: three counter passes (SQ set, FETCH_SIZE,
# WRITE_SIZE), each its own rocprofv3 run with --kernel-trace only, then merged per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
NAME=sq T=300 bash scripts/pmc_session.sh || exit $?
CTRS="FETCH_SIZE" NAME=fetch T=300 bash scripts/pmc_session.sh || exit $?
CTRS="WRITE_SIZE" NAME=write T=300 bash scripts/pmc_session.sh || exit $?
find gpurun_out/pmc -name "*counter_collection.csv" | sort
sq=$(find gpurun_out/pmc -name "sq*counter_collection.csv" | head -1)
fe=$(find gpurun_out/pmc -name "fetch*counter_collection.csv" | head -1)
wr=$(find gpurun_out/pmc -name "write*counter_collection.csv" | head -1)
python3 scripts/pmc_merge.py "$sq" "$fe" "$wr" > gpurun_out/pmc/merged.md
head -24 gpurun_out/pmc/merged.md
