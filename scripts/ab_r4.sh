#!/bin/bash
# Round-4 build (ab_r4/: its bench, package and library, gitignored) against HEAD on one
# box, alternating: C3 and C2 V-cycles/s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for p in 27pt 7pt; do
  for i in 1 2; do
    timeout -k 10 300 python3 ab_r4/bench.py --problem $p --steps 50 --warmup 3 --no-cpu-baseline --no-general --no-abi \
        > gpurun_out/r4_${p}_$i.json 2> gpurun_out/r4_${p}_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --problem $p --steps 50 --warmup 3 --no-cpu-baseline --no-general --no-abi \
        > gpurun_out/head_${p}_$i.json 2> gpurun_out/head_${p}_$i.err || exit 1
    echo "$p rep $i r04 $(grep -o '"value": [0-9.]*' gpurun_out/r4_${p}_$i.json) HEAD $(grep -o '"value": [0-9.]*' gpurun_out/head_${p}_$i.json)"
  done
done
