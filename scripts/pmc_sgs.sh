#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the fused 27-point SGS
# phases of scripts/time_sgs.py: SQ cycle buckets, instruction mix, HBM bytes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MODES=1
R=$(pwd)
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d "$R/gpurun_out/pmc_sgs$i" -o run --output-format csv \
      -- python3 "$R/scripts/time_sgs.py" > "$R/gpurun_out/pmc_sgs$i.log" 2>&1 || exit 1
done
