#!/bin/bash
# k_fine_rr (v2) vs the round-5 resid+restrict kernel: bitwise test, then timing A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "fine_fused" > gpurun_out/r6_rr2_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r6_rr2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/time_fused.py 0 1 2 3 > gpurun_out/r6_rr2_time.log 2>&1 || exit $?
FAMG_FINE_RR=1 FAMG_FINE_PJ=1 timeout -k 10 200 python scripts/time_fused.py 0 > gpurun_out/r6_rr1_time.log 2>&1 || exit $?
tail -1 gpurun_out/r6_rr2_time.log; tail -1 gpurun_out/r6_rr1_time.log
