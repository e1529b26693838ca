#!/bin/bash
# Setup-time tile decisions of every benchmark configuration, timed
# (FAMG_TUNE_RETIME=1 ignores the frozen table) -> gpurun_out/tuning_log.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FAMG_TUNE_RETIME=1 FAMG_TUNE_LOG="$(pwd)/gpurun_out/tuning_log.txt"
mkdir -p gpurun_out
rm -f "$FAMG_TUNE_LOG"
B="--steps 2 --warmup 1 --no-cpu-baseline --no-general --no-abi"
timeout -k 10 300 python3 bench.py $B > gpurun_out/tc_c2.json 2> gpurun_out/tc_c2.err || exit 1
timeout -k 10 300 python3 bench.py --problem 27pt $B > gpurun_out/tc_c3.json 2> gpurun_out/tc_c3.err || exit 1
timeout -k 10 300 python3 bench.py --problem elast $B > gpurun_out/tc_c5.json 2> gpurun_out/tc_c5.err || exit 1
for n in 2 4 8; do
  timeout -k 10 600 python3 bench.py --loopback $n $B > gpurun_out/tc_lb$n.json 2> gpurun_out/tc_lb$n.err || exit 1
done
