#!/bin/bash
# C5: 3x3-block kernel choices for the fine level, alternating on one box:
# default | one-wave workgroups everywhere | the round-2 kernel on A_0 (long-row threshold 48)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  for v in def ow long48; do
    case $v in def) E="";; ow) E="FAMG_BSR_ONE_WAVE=1000000";; long48) E="FAMG_BSR_LONG=48";; esac
    env $E timeout -k 10 200 python3 bench.py --problem elast --steps 100 --warmup 5 --no-cpu-baseline --no-general \
        --no-abi > gpurun_out/c5b_${v}_$i.json 2> gpurun_out/c5b_${v}_$i.err || exit 1
    echo "$v rep $i $(grep -o '"value": [0-9.]*' gpurun_out/c5b_${v}_$i.json)"
  done
done
