#!/bin/bash
# Wave-state and cache counters of the C5 fine-level 3x3-block SpMV
# (scripts/pmc_bsr.py: CAL block-diagonal launches, then the elasticity
# operator), one counter group per rocprofv3 pass -> gpurun_out/pmc_bsrq*/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace -d "$R/gpurun_out/pmc_bsrq$i" -o run --output-format csv \
      -- python3 "$R/scripts/pmc_bsr.py" > "$R/gpurun_out/pmc_bsrq$i.log" 2>&1 || exit 1
done
