#!/bin/bash
# PMC passes (one counter group per run) over scripts/pmc_xscs.py: cache and
# wave-state counters of the x-staged stencil-class kernels on A_1..A_3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FAMG_XSCS_VS_DIA=1  # A_1 as classes (not timed against DIA)
R=$(pwd)
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace -d "$R/gpurun_out/pmc_xscs$i" -o run --output-format csv \
      -- python3 "$R/scripts/pmc_xscs.py" > "$R/gpurun_out/pmc_xscs$i.log" 2>&1 || exit 1
done
python3 scripts/pmc_xscs_summary.py gpurun_out > gpurun_out/pmc_xscs_summary.json
