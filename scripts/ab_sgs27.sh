cd $GRAFT_REPO_ROOT; for t in 16 16; do FAMG_SGS27_TY=$t timeout -k 10 120 python scripts/time_sgs.py 2>/dev/null || exit 1; done
