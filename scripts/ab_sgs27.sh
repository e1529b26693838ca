#!/bin/bash
# A/B of the fused SGS phase kernel variants (each in its own process: the
# switches are read once)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python scripts/time_sgs.py 2>/dev/null || exit 1
for v in "FAMG_SGS27_OL=0" "FAMG_SGS27_OL=0 FAMG_SGS27_TY=32 FAMG_SGS27_NW=8" "FAMG_SGS27_CST=0"; do
  env $v MODES=1,2 timeout -k 10 120 python scripts/time_sgs.py 2>/dev/null || exit 1
done
