#!/bin/bash
# C5 stand-in, round-2 build (ab_r2/: its bench, package and library, gitignored)
# against HEAD on one box, alternating: V-cycles/s and the hierarchy of each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python3 ab_r2/bench.py --problem elast --steps 30 --warmup 3 --no-cpu-baseline --no-general \
      > gpurun_out/c5_r2_$i.json 2> gpurun_out/c5_r2_$i.err || exit 1
  timeout -k 10 200 python3 bench.py --problem elast --steps 30 --warmup 3 --no-cpu-baseline --no-general --no-abi \
      > gpurun_out/c5_head_$i.json 2> gpurun_out/c5_head_$i.err || exit 1
done
for k in 0 1 2 3; do
  FAMG_BSR_KERNEL=$k timeout -k 10 200 python3 bench.py --problem elast --steps 30 --warmup 3 --no-cpu-baseline \
      --no-general --no-abi > gpurun_out/c5_bsr$k.json 2> gpurun_out/c5_bsr$k.err || exit 1
done
