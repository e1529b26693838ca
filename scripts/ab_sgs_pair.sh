#!/bin/bash
# C3: round-4 build vs HEAD with the marching SGS colour pairs off / on, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 ab_r4/bench.py --problem 27pt --steps 50 --warmup 3 --no-cpu-baseline --no-general --no-abi \
      > gpurun_out/sp_r4_$i.json 2> gpurun_out/sp_r4_$i.err || exit 1
  for p in 0 1; do
    FAMG_SGS27_PAIR=$p timeout -k 10 300 python3 bench.py --problem 27pt --steps 50 --warmup 3 --no-cpu-baseline --no-general \
        --no-abi > gpurun_out/sp_head${p}_$i.json 2> gpurun_out/sp_head${p}_$i.err || exit 1
  done
  echo "rep $i r04 $(grep -o '"value": [0-9.]*' gpurun_out/sp_r4_$i.json) HEAD pair0 $(grep -o '"value": [0-9.]*' gpurun_out/sp_head0_$i.json) pair1 $(grep -o '"value": [0-9.]*' gpurun_out/sp_head1_$i.json)"
done
