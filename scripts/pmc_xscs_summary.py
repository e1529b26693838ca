"""Per-kernel medians of the PMC passes of scripts/pmc_xscs.sh (the 10 SET
launches of A_1, A_2, A_3 in dispatch order).  FETCH_SIZE is KiB as reported
(uncalibrated for this gather pattern; MI355X_MICROARCH.md HBM section)."""
import csv
import glob
import json
import os
import statistics
import sys

out_dir = sys.argv[1]
per = {}
for f in sorted(glob.glob(os.path.join(out_dir, "pmc_xscs*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "xscs" not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Counter_Name"], []).append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
res = {}
for ctr, vals in per.items():
    vals.sort()
    vals = vals[-30:]  # the workload's launches (setup autotuning also launches xscs kernels)
    for lvl in range(3):
        chunk = vals[10 * lvl:10 * lvl + 10]
        if not chunk:
            continue
        d = res.setdefault("A_%d" % (lvl + 1), {"kernel": chunk[0][1]})
        d[ctr] = statistics.median(v for _, _, v in chunk)
for d in res.values():
    h, m = d.get("TCC_HIT_sum"), d.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        d["L2_hit_rate"] = round(h / (h + m), 4)
    w = d.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in d:
                d[k + "_frac"] = round(d[k] / w, 4)
print(json.dumps(res, indent=1))
