#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over scripts/pmc_bsr_renum.py, then the summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmcb_fetch" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_bsr_renum.py" > "$R/gpurun_out/pmcb_fetch.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmcb_write" -o run --output-format csv \
    -- python3 "$R/scripts/pmc_bsr_renum.py" > "$R/gpurun_out/pmcb_write.log" 2>&1 || exit 1
python3 - "$R" <<'PY'
import csv, glob, json, os, statistics, sys
R = sys.argv[1]
known = json.load(open(os.path.join(R, "gpurun_out", "pmc_bsr_renum_known.json")))
it = known["iters"]
def load(d, counter):
    path = sorted(glob.glob(os.path.join(R, "gpurun_out", d, "**", "*counter_collection.csv"), recursive=True))[0]
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and "spmv_bsr3" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    v = [float(r["Counter_Value"]) * 1024.0 for r in rows][-2 * it:]
    return v[:it], v[it:], rows[-1]["Kernel_Name"].split("(")[0]
cf, ff, kname = load("pmcb_fetch", "FETCH_SIZE")
cw, fw, _ = load("pmcb_write", "WRITE_SIZE")
factor = (known["cal_alg"] - 8 * known["n"]) / statistics.median(cf)
rd = statistics.median(ff) * factor
wr = statistics.median(fw)
out = {"workload": "C5 stand-in fine SpMV as the cycle runs it (locality-renumbered copy), SET",
       "kernel": kname, "fetch_correction_factor": round(factor, 4),
       "calibration": {"known_read_bytes": known["cal_alg"] - 8 * known["n"], "fetch_size_bytes": statistics.median(cf),
                       "write_size_bytes": statistics.median(cw), "known_write_bytes": 8 * known["n"]},
       "algorithmic_bytes_per_launch": known["fine_alg"], "read_bytes_per_launch": round(rd),
       "write_bytes_per_launch": round(wr), "hbm_bytes_per_launch": round(rd + wr),
       "ratio": round((rd + wr) / known["fine_alg"], 4)}
json.dump(out, open(os.path.join(R, "gpurun_out", "c5_renum_spmv_traffic.json"), "w"), indent=1)
print(json.dumps(out))
PY
