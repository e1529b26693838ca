#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over scripts/pmc_cycle.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmcc_fetch" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_cycle.py" > "$R/gpurun_out/pmcc_fetch.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmcc_write" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_cycle.py" > "$R/gpurun_out/pmcc_write.log" 2>&1 || exit 1
python3 scripts/pmc_cycle_summary.py gpurun_out/pmcc_fetch \
    gpurun_out/pmcc_write gpurun_out/pmc_cycle_known.json gpurun_out/pmc_cycle_plan.json \
    gpurun_out/c2_cycle_traffic.json
