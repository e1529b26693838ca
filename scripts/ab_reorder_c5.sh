#!/bin/bash
# C5 stand-in with the locality renumbering off / auto, alternating on one box
# (V-cycles/s), then one kernel trace of each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  for r in 0 1; do
    timeout -k 10 200 python3 bench.py --problem elast --steps 100 --warmup 5 --no-cpu-baseline --no-general \
        --no-abi --reorder $r > gpurun_out/c5_reorder${r}_$i.json 2> gpurun_out/c5_reorder${r}_$i.err || exit 1
    echo "reorder=$r rep=$i $(grep -o '"value": [0-9.]*' gpurun_out/c5_reorder${r}_$i.json) $(grep -o '"locality_renumbered_levels": [^]]*]' gpurun_out/c5_reorder${r}_$i.json)"
  done
done
C5_ARGS="--reorder 0" bash scripts/prof_c5.sh c5_reorder0 > /dev/null || exit 1
C5_ARGS="--reorder 1" bash scripts/prof_c5.sh c5_reorder1 > /dev/null || exit 1
grep -E "per V-cycle|^ +[0-9]+ +0 " gpurun_out/c5_reorder0.txt gpurun_out/c5_reorder1.txt
