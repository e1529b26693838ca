#!/bin/bash
# A/B of round-3 switches on the C2 bench (one process per setting, 50 cycles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run NAME ENV...
    local name=$1; shift
    env "$@" timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-general \
        > "gpurun_out/ab_$name.log" 2>&1 || { echo "$name failed rc=$?"; exit 1; }
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$name.log)"
}
run base FAMG_FOLD_XSCS=1
run nofold FAMG_FOLD_XSCS=0
run wpr1 FAMG_VEC_WPR=1
run wpr2 FAMG_VEC_WPR=2
run base2 FAMG_FOLD_XSCS=1
