#!/bin/bash
# rocprofv3 kernel trace of the C2 bench (20 cycles) into gpurun_out/$1 with its
# launch plan; extra environment (A/B switches) from the caller
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$1" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-general --no-abi --no-secondary --plan-out "$R/gpurun_out/$1.plan.json" \
    > "$R/gpurun_out/$1.log" 2>&1 || exit $?
python3 scripts/prof_summary.py --steps 20 --plan "gpurun_out/$1.plan.json" "gpurun_out/$1/run_kernel_trace.csv" > "gpurun_out/$1.txt"
grep -E "gtc|per V-cycle" "gpurun_out/$1.txt"
