"""Per-kernel medians of the counter passes of scripts/pmc_fused.sh (fused
fine-level kernels), FETCH_SIZE (KiB, x2: the gfx950 correction of
MI355X_MICROARCH.md) + WRITE_SIZE as HBM bytes per launch."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    out = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("famg::", "")
        if "k_fine" not in k:
            continue
        out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


agg = defaultdict(dict)
for d in sys.argv[1:]:
    for k, cs in load(d).items():
        for c, v in cs.items():
            agg[k][c] = statistics.median(v)
for k, cs in agg.items():
    print(k)
    for c in sorted(cs):
        print(f"  {c:28s} {cs[c]:16.1f}")
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        print(f"  HBM bytes per launch (2 x FETCH + WRITE): {(2 * cs['FETCH_SIZE'] + cs['WRITE_SIZE']) * 1024 / 1e6:.1f} MB")
    if "SQ_WAVE_CYCLES" in cs:
        w = cs["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in cs:
                print(f"  {c} / WAVE_CYCLES = {cs[c] / w:.3f}")
