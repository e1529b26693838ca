#!/bin/bash
# C5 stand-in with the long-row 3x3-block kernel threshold (FAMG_BSR_LONG) varied,
# alternating on one box: V-cycles/s per setting and repetition
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  for t in -1 16 48 0; do
    FAMG_BSR_LONG=$t timeout -k 10 200 python3 bench.py --problem elast --steps 200 --warmup 5 --no-cpu-baseline \
        --no-general --no-abi > gpurun_out/c5_long${t}_$i.json 2> gpurun_out/c5_long${t}_$i.err || exit 1
    echo "long=$t rep=$i $(grep -o '"value": [0-9.]*' gpurun_out/c5_long${t}_$i.json)"
  done
done
