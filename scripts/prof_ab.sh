#!/bin/bash
# rocprofv3 kernel traces of the default bench with and without an env switch:
#   bash scripts/prof_ab.sh NAME VAR=VALUE   -> gpurun_out/prof_NAME_{a,b}
# (BENCH_ARGS overrides the bench arguments, e.g. "--problem 27pt --smoother sgs")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); name=$1; shift
BA=${BENCH_ARGS:-"--steps 20 --warmup 3"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${name}_a" -o run --output-format csv \
    -- python3 "$R/bench.py" $BA --no-cpu-baseline --no-general > "$R/gpurun_out/prof_${name}_a.log" 2>&1 &&
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${name}_b" -o run --output-format csv \
    -- python3 "$R/bench.py" $BA --no-cpu-baseline --no-general > "$R/gpurun_out/prof_${name}_b.log" 2>&1
