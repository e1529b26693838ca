set -e
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -n 1 gpurun_out/t_all.log
run() {
MODES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/m_$1 -o run --output-format csv -- python3 scripts/time_sgs.py > gpurun_out/m_$1.log 2>&1
python3 - <<PY
import csv
rows=[r for r in csv.DictReader(open("gpurun_out/m_$1/run_kernel_trace.csv")) if "sgs27_" in r["Kernel_Name"]]
d=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in rows]
ph=[sorted(d[k::4])[len(d[k::4])//2] for k in range(4)]
print("$1", rows[-1]["Kernel_Name"][:36], ["%.1f"%x for x in ph], "%.1f" % sum(ph))
PY
}
FAMG_SGS27_MARCH=0 run off
FAMG_SGS27_MARCH=1 run auto16
FAMG_SGS27_MARCH=4 run j4_16
FAMG_SGS27_MNW=8 FAMG_SGS27_MARCH=1 run auto8
FAMG_SGS27_MNW=8 FAMG_SGS27_MARCH=4 run j4_8
FAMG_BSR_X16=0 bash scripts/prof_c5.sh c5x0
FAMG_BSR_X16=1 bash scripts/prof_c5.sh c5x1
