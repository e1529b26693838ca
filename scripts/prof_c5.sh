#!/bin/bash
# rocprofv3 kernel trace of the C5 stand-in bench (20 cycles) into gpurun_out/$1 ($C5_ARGS: extra bench arguments)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$1" -o run --output-format csv \
    -- python3 "$R/bench.py" --problem elast --steps 20 --warmup 3 --no-cpu-baseline --no-abi --no-general $C5_ARGS \
    --plan-out "$R/gpurun_out/$1.plan.json" \
    > "$R/gpurun_out/$1.log" 2>&1 || exit $?
python3 scripts/prof_summary.py --steps 20 --plan "gpurun_out/$1.plan.json" "gpurun_out/$1/run_kernel_trace.csv" > "gpurun_out/$1.txt"
grep -E "bsr3|per V-cycle" "gpurun_out/$1.txt"
grep -E '"value"' "gpurun_out/$1.log" | cut -c1-200
