#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over scripts/pmc_cycle.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
# the dense tail's one-time build (4096 eager sub-cycles, ~30K dispatches) crashed
# rocprofv3's counter collection (SIGSEGV in a dispatch, round 6): the counted
# cycle runs every level (the fine-level launches are the same either way)
export FAMG_DENSE_TAIL=0
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmcc_fetch" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_cycle.py" > "$R/gpurun_out/pmcc_fetch.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmcc_write" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_cycle.py" > "$R/gpurun_out/pmcc_write.log" 2>&1 || exit 1
python3 scripts/pmc_cycle_summary.py gpurun_out/pmcc_fetch \
    gpurun_out/pmcc_write gpurun_out/pmc_cycle_known.json gpurun_out/pmc_cycle_plan.json \
    gpurun_out/c2_cycle_traffic.json
