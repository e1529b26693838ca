cd $GRAFT_REPO_ROOT
for v in "16 1 0" "12 1 0" "8 1 0" "24 1 0" "16 1 6"; do
  set -- $v
  FAMG_SGS27_TY=$1 FAMG_SGS27_U=$2 FAMG_SGS27_DEBUG=$3 timeout -k 10 120 python scripts/time_sgs.py 2>/dev/null | sed "s/^/dbg=$3 /" || exit 1
done
