#!/bin/bash
# One SQ counter pass over the C2 bench (few cycles): LDS conflicts and wait
# buckets of the grid-transfer kernels (k_gtc_*); summary by kernel name
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
    --kernel-trace -d "$R/gpurun_out/pmc_gtc" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-general --no-abi > "$R/gpurun_out/pmc_gtc.log" 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob("gpurun_out/pmc_gtc/**/*counter_collection.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0]
        if "gtc" not in n and "dia_kernel" not in n:
            continue
        per[n][r["Counter_Name"]] += float(r["Counter_Value"])
        k = (n, r["Dispatch_Id"])
        if k not in seen:
            seen.add(k); cnt[n] += 1
for n, d in per.items():
    w = d.get("SQ_WAVE_CYCLES", 1)
    act = d.get("SQ_LDS_IDX_ACTIVE", 0)
    print(n, "launches", cnt[n], "lds_conflict_frac %.3f" % (d.get("SQ_LDS_BANK_CONFLICT", 0) / max(act, 1)),
          "wait_any %.3f" % (d.get("SQ_WAIT_ANY", 0) / w), "wait_inst %.3f" % (d.get("SQ_WAIT_INST_ANY", 0) / w),
          "wait_inst_lds %.3f" % (d.get("SQ_WAIT_INST_LDS", 0) / w), "lds_insts/wave %.0f" % (d.get("SQ_INSTS_LDS", 0) / max(d.get("SQ_WAVES", 1), 1)))
PY
