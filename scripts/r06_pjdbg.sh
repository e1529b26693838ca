#!/bin/bash
# k_fine_pj timing with parts switched off (FAMG_FINE_DBG bits: 1 no stores, 2 no P sums, 4 no Jacobi sums)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/time_fused.py 0 1 2 4 6 7 > gpurun_out/r6_pjdbg.log 2>&1 || exit $?
tail -1 gpurun_out/r6_pjdbg.log
