set -e
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/benchprof" -o run --output-format csv -- python3 "$R/bench.py" > gpurun_out/benchprof.log 2>&1 || { tail -20 gpurun_out/benchprof.log; exit 1; }
grep '^{' gpurun_out/benchprof.log | cut -c1-200
bash scripts/prof_dist1.sh dist1r4
grep '^{' gpurun_out/dist1r4.log | cut -c1-250
