#!/bin/bash
# Round-end evidence on one MI355X, into gpurun_out/final/: the driver's default
# bench line, the same command under rocprofv3 --kernel-trace --stats (the
# roofline kernel's average duration must agree with the line's ms_per_launch),
# the C3 / C5 lines with cpu_baseline and parity, and the 1-rank distributed line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p "$O"
# heartbeat: the CPU baseline / parity legs of the C3 / C5 lines run minutes without output
( while sleep 50; do date >> "$O/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
SKIP=${SKIP:-}
[[ $SKIP == *bench* ]] || timeout -k 10 400 python3 bench.py > "$O/bench_stdout.log" 2> "$O/bench_stderr.log" || exit 1
echo "bench: $(tail -1 "$O/bench_stdout.log" | cut -c1-160)"
[[ $SKIP == *prof* ]] || timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" > "$O/bench_prof_stdout.log" 2> "$O/bench_prof_stderr.log" || exit 1
echo "bench under rocprofv3: $(tail -1 "$O/bench_prof_stdout.log" | cut -c1-160)"
timeout -k 10 500 python3 bench.py --problem 27pt > "$O/c3_stdout.log" 2> "$O/c3_stderr.log" || exit 1
echo "c3: $(tail -1 "$O/c3_stdout.log" | cut -c1-160)"
timeout -k 10 500 python3 bench.py --problem elast > "$O/c5_stdout.log" 2> "$O/c5_stderr.log" || exit 1
echo "c5: $(tail -1 "$O/c5_stdout.log" | cut -c1-160)"
timeout -k 10 500 python3 bench.py --dist > "$O/dist1_stdout.log" 2> "$O/dist1_stderr.log" || exit 1
echo "dist1: $(tail -1 "$O/dist1_stdout.log" | cut -c1-160)"
