#!/bin/bash
# PMC HBM traffic of roofline.csr's SpMV (the x-staged SELL kernel on the random
# 7-pt 256^3 operator, window 4096): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (MI355X_MICROARCH.md), FETCH calibrated on a permutation
# matrix through the same kernel -> gpurun_out/csr_spmv_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_csr_f" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_general.py" xsell > "$R/gpurun_out/pmc_csr_f.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_csr_w" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_general.py" xsell > "$R/gpurun_out/pmc_csr_w.log" 2>&1 &&
python3 scripts/pmc_general_summary.py $(find gpurun_out/pmc_csr_f -name "*counter_collection.csv" | head -1) \
    $(find gpurun_out/pmc_csr_w -name "*counter_collection.csv" | head -1) gpurun_out/pmc_general_known_xsell.json \
    gpurun_out/csr_spmv_traffic.json
