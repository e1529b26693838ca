#!/bin/bash
# rocprofv3 kernel trace of the distributed bench at world size 1 (one RCCL
# rank, run directly: no launcher hop under the profiler) into gpurun_out/$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$1" -o run --output-format csv \
    -- python3 "$R/bench.py" --dist --steps 20 --warmup 3 --plan-out "$R/gpurun_out/$1.plan.json" ${@:2} \
    > "$R/gpurun_out/$1.log" 2>&1 || exit $?
python3 scripts/prof_summary.py --steps 20 --plan "gpurun_out/$1.plan.json" "gpurun_out/$1/run_kernel_trace.csv" > "gpurun_out/$1.txt"
grep -E "per V-cycle" "gpurun_out/$1.txt"
