"""Per-launch SQ counters of the C2 cycle (scripts/pmc_cycle_sq.sh): the
dispatches between k_trace_mark<<<1>>> and <<<2>>> matched to the launch plan
position by position, medians over the cycles.

  python scripts/pmc_cycle_sq.py COUNTER_DIR PLAN.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main(d, plan_json):
    plan = json.load(open(plan_json))
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    by = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        i = int(r["Dispatch_Id"])
        by[i][r["Counter_Name"]] = by[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    ids = sorted(by)
    marks = [i for i in ids if "k_trace_mark" in names[i]]
    cyc = [i for i in ids if marks[-2] < i < marks[-1]]
    n = len(plan)
    assert len(cyc) % n == 0, (len(cyc), n)
    print(f"{'#':>3} {'lvl':>3} {'role':8} {'storage':10} {'waves':>7} {'VALU/w':>7} {'LDS/w':>6} "
          f"{'wait':>5} {'winst':>5} {'active':>6} {'busy%':>5}  kernel")
    for k, p in enumerate(plan):
        rows = [by[cyc[c * n + k]] for c in range(len(cyc) // n)]
        med = {c: statistics.median(r.get(c, 0.0) for r in rows) for c in rows[0]}
        w = max(med.get("SQ_WAVES", 1.0), 1.0)
        wc = max(med.get("SQ_WAVE_CYCLES", 1.0), 1.0)
        kname = names[cyc[k]].split("(")[0].replace("void ", "").replace("famg::", "")[:48]
        print(f"{k:3d} {p['level']:3d} {p.get('role', ''):8s} {p.get('name', ''):10s} {int(w):7d} "
              f"{med.get('SQ_INSTS_VALU', 0) / w:7.0f} {med.get('SQ_INSTS_LDS', 0) / w:6.0f} "
              f"{med.get('SQ_WAIT_ANY', 0) / wc:5.2f} {med.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"{med.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.2f} {100 * med.get('SQ_BUSY_CYCLES', 0) / max(med.get('SQ_BUSY_CYCLES', 1), 1):5.0f}  {kname}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
