#!/bin/bash
# A_3 of the C2 cycle: x-staged classes (default) vs the lanes-per-row class kernel (FAMG_SCS_ROWS=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/prof_c2.sh r6_ab_base > /dev/null || exit $?
FAMG_SCS_ROWS=1 bash scripts/prof_c2.sh r6_ab_rows > /dev/null || exit $?
for t in base rows; do echo "== $t"; grep "per V-cycle" gpurun_out/r6_ab_$t.txt | head -1; grep -E "^ +[0-9]+ +3 " gpurun_out/r6_ab_$t.txt; done
