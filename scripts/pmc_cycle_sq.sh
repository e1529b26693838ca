#!/bin/bash
# one SQ-counter pass over scripts/pmc_cycle.py: per launch of the C2 cycle the
# wave count, instruction mix and wait fractions (scripts/pmc_cycle_sq.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
# (the dense tail's one-time build under counter collection crashed rocprofv3: scripts/pmc_cycle.sh)
export FAMG_DENSE_TAIL=0
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d "$R/gpurun_out/pmcc_sq" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_cycle.py" > "$R/gpurun_out/pmcc_sq.log" 2>&1 || exit 1
python3 scripts/pmc_cycle_sq.py gpurun_out/pmcc_sq gpurun_out/pmc_cycle_plan.json > gpurun_out/pmc_cycle_sq.txt
cat gpurun_out/pmc_cycle_sq.txt
