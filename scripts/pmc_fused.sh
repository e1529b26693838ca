#!/bin/bash
# wave-state / LDS / memory counters of the fused fine-level kernels, one
# counter group per rocprofv3 pass -> gpurun_out/pmc_fused*/ + summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
# (the dense tail's one-time build under counter collection crashed rocprofv3: scripts/pmc_cycle.sh)
export FAMG_DENSE_TAIL=0
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace -d "$R/gpurun_out/pmc_fused$i" -o run --output-format csv \
      -- python3 "$R/scripts/pmc_fused.py" > "$R/gpurun_out/pmc_fused$i.log" 2>&1 || exit 1
done
python3 scripts/pmc_fused_summary.py gpurun_out/pmc_fused1 gpurun_out/pmc_fused2 gpurun_out/pmc_fused3 gpurun_out/pmc_fused4 \
    > gpurun_out/pmc_fused_summary.txt
cat gpurun_out/pmc_fused_summary.txt
