"""Per-phase medians of the PMC passes of scripts/pmc_sgs.sh: the fused SGS
phase launches of scripts/time_sgs.py (MODES=1, four phases per step, phase k =
launch index mod 4).  FETCH_SIZE / WRITE_SIZE in KiB as reported; the HBM
bytes quoted in DESIGN.md apply the fetch calibration of
profiles/r04/c2_cycle_traffic.json."""
import csv
import glob
import json
import os
import statistics
import sys

out_dir = sys.argv[1]
per = {}
for f in sorted(glob.glob(os.path.join(out_dir, "pmc_sgs*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "k_sgs27_phase" not in r["Kernel_Name"] and "k_sgs27_march" not in r["Kernel_Name"]:
            continue
        key = (os.path.dirname(f), int(r["Dispatch_Id"]))
        per.setdefault(r["Counter_Name"], {}).setdefault(key, [r["Kernel_Name"], 0.0])[1] += float(r["Counter_Value"])
res = {}
for ctr, disp in per.items():
    vals = [disp[k] for k in sorted(disp)]
    for ph in range(4):
        chunk = vals[ph::4]
        if not chunk:
            continue
        d = res.setdefault("phase_%d" % ph, {"kernel": chunk[0][0], "launches": len(chunk)})
        d[ctr] = statistics.median(v for _, v in chunk)
for d in res.values():
    w = d.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if k in d:
                d[k + "_frac"] = round(d[k] / w, 4)
    if d.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_frac"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"], 4)
    if d.get("FETCH_SIZE") is not None:
        d["fetch_MB"] = round(d["FETCH_SIZE"] * 1024 / 1e6, 2)
    if d.get("WRITE_SIZE") is not None:
        d["write_MB"] = round(d["WRITE_SIZE"] * 1024 / 1e6, 2)
print(json.dumps(res, indent=1))
