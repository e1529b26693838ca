#!/bin/bash
# fused fine-level kernels, coarse solve, SpMM: parity tests, then the C2 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "fine_fused or cycle_plan_accounts or constant_diagonal or dia7_row or storage_mix or setdf or gtc or coarse_cholesky or spmm" > gpurun_out/r6_fuse_pytest.log 2>&1
rc=$?; tail -25 gpurun_out/r6_fuse_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/prof_c2.sh r6_c2f > /dev/null; head -12 gpurun_out/r6_c2f.txt; grep -A25 "per launch" gpurun_out/r6_c2f.txt
timeout -k 10 300 python scripts/time_spmm.py > gpurun_out/spmm_timing.log 2>&1; tail -8 gpurun_out/spmm_timing.log
