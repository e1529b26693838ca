#!/bin/bash
# rocprofv3 kernel trace of the C3 bench (10 cycles) into gpurun_out/$1 with its launch plan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$1" -o run --output-format csv \
    -- python3 "$R/${BENCH:-bench.py}" --problem 27pt --steps 10 --warmup 2 --no-cpu-baseline --no-general --no-abi \
    --plan-out "$R/gpurun_out/$1.plan.json" > "$R/gpurun_out/$1.log" 2>&1 || exit $?
python3 scripts/prof_summary.py --steps 10 --plan "gpurun_out/$1.plan.json" "gpurun_out/$1/run_kernel_trace.csv" > "gpurun_out/$1.txt"
grep -E "per V-cycle| 1 (restrict|interp) " "gpurun_out/$1.txt"
