set -e
export TMPDIR=/tmp
FAMG_BSR_LATE=1 bash scripts/prof_c5.sh c5late > /dev/null; grep -E "bsr3|per V-cycle" gpurun_out/c5late.txt | head -8; grep -o '"value": [0-9.]*' gpurun_out/c5late.log | head -1
FAMG_BSR_LATE=0 bash scripts/prof_c5.sh c5early > /dev/null; grep -E "bsr3|per V-cycle" gpurun_out/c5early.txt | head -8; grep -o '"value": [0-9.]*' gpurun_out/c5early.log | head -1
