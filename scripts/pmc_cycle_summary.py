"""HBM traffic per launch of the C2 cycle from the FETCH_SIZE / WRITE_SIZE
passes over scripts/pmc_cycle.py, against the launch plan's algorithmic bytes.

  python scripts/pmc_cycle_summary.py FETCH_DIR WRITE_DIR KNOWN.json PLAN.json OUT.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  The first ITERS DIA dispatches
are the calibration (diagonal matrix: 4 n code bytes + 8 n read, 8 n written),
the next ITERS the fine SET SpMV, then the CYCLES cycles between the trace marks
(matched to the plan position by position).  Read bytes = FETCH_SIZE x the
calibration factor (~2 on gfx950 for 16-B/lane streams); other access widths
are reported with the same factor and their raw value beside it.
"""
import csv
import json
import statistics
import sys


def load(path, counter):
    import glob
    import os
    if os.path.isdir(path):  # rocprofv3 -d DIR: the counter CSV may sit in a per-process subdirectory
        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[0]
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0, int(r["Grid_Size"]) if "Grid_Size" in r else 0)
            for r in rows]


def split(rows, iters, cycles, nplan):
    names = [r[0] for r in rows]
    marks = [i for i, nm in enumerate(names) if "k_trace_mark" in nm]
    assert len(marks) >= 2, "no trace marks"
    cp, lo = [], 0
    if len(marks) >= 4:  # marks 3, 4 bracket the torch copies, then 1, 2 the cycles
        cp = list(range(marks[0] + 1, marks[1]))
        lo, marks = marks[1] + 1, marks[2:]
    # CAL and FINE sit between the copy marks and the cycle marks (the warm-up
    # cycle before the copies also runs DIA kernels and must not be counted)
    dia = [i for i in range(lo, marks[0]) if "spmv_dia_kernel" in names[i] or "spmv_dia7c_kernel" in names[i]]
    cal, fine = dia[:iters], dia[iters:2 * iters]
    cyc = list(range(marks[0] + 1, marks[1]))
    assert len(cyc) == cycles * nplan, (len(cyc), cycles, nplan)
    return cal, fine, cyc, cp


def main(fetch_csv, write_csv, known_json, plan_json, out_json):
    known = json.load(open(known_json))
    plan = json.load(open(plan_json))
    n, iters, cycles = known["n"], known["iters"], known["cycles"]
    F, W = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    cal, fine, cyc, cp = split(F, iters, cycles, len(plan))
    calw, finew, cycw, cpw = split(W, iters, cycles, len(plan))
    cal_known = known["cal"]["stream_bytes"] + 8 * n
    dia_factor = cal_known / statistics.median(F[i][1] for i in cal)
    copy = None
    if cp:  # the 16-B/lane copy calibration is the one used when present
        factor = 8 * n / statistics.median(F[i][1] for i in cp)
        copy = {"kernel": F[cp[0]][0].split("(")[0][:80], "known_read_bytes": 8 * n,
                "fetch_size_bytes": statistics.median(F[i][1] for i in cp),
                "write_size_bytes": statistics.median(W[i][1] for i in cpw), "known_write_bytes": 8 * n,
                "factor": round(factor, 4)}
    else:
        factor = dia_factor
    fine_alg = known["fine"]["stream_bytes"] + 16 * n
    fine_rd = statistics.median(F[i][1] for i in fine) * factor
    fine_wr = statistics.median(W[i][1] for i in finew)
    launches = []
    for p, rec in enumerate(plan):
        rd = statistics.median(F[cyc[c * len(plan) + p]][1] for c in range(cycles))
        wr = statistics.median(W[cycw[c * len(plan) + p]][1] for c in range(cycles))
        kname = F[cyc[p]][0].split("(")[0].replace("void ", "").replace("famg::", "")
        hbm = rd * factor + wr
        launches.append({"pos": p, "level": rec["level"], "role": rec["role"], "storage": rec["name"],
                         "mode": rec["mode"], "kernel": kname, "algorithmic_bytes": rec["bytes"],
                         "fetch_size_raw": round(rd), "write_size": round(wr), "hbm_bytes": round(hbm),
                         "ratio": round(hbm / max(1, rec["bytes"]), 4)})
    out = {
        "workload": "C2 hierarchy (7-pt 256^3, SA 2^3 boxes), eager V-cycles; FETCH/WRITE passes separate",
        "fetch_correction_factor": round(factor, 4),
        "copy_calibration": copy,
        "calibration": {"factor": round(dia_factor, 4), "kernel": "spmv_dia_kernel<SET> on a diagonal matrix (4-bit DIA codes)",
                        "known_read_bytes": cal_known,
                        "fetch_size_bytes": statistics.median(F[i][1] for i in cal),
                        "write_size_bytes": statistics.median(W[i][1] for i in calw), "known_write_bytes": 8 * n},
        "fine_set": {"kernel": F[fine[0]][0].split("(")[0].replace("void ", "").replace("famg::", "") + " on A_0 (7-pt 256^3)",
                     "algorithmic_bytes_per_launch": fine_alg,
                     "read_bytes_per_launch": round(fine_rd), "write_bytes_per_launch": round(fine_wr),
                     "hbm_bytes_per_launch": round(fine_rd + fine_wr),
                     "ratio": round((fine_rd + fine_wr) / fine_alg, 4)},
        "cycle_hbm_bytes": round(sum(l["hbm_bytes"] for l in launches)),
        "cycle_algorithmic_bytes": sum(l["algorithmic_bytes"] for l in launches),
        "launches": launches,
    }
    json.dump(out, open(out_json, "w"), indent=1)
    print(f"factor {factor:.4f}; fine SET {out['fine_set']['ratio']}; cycle "
          f"{out['cycle_hbm_bytes'] / out['cycle_algorithmic_bytes']:.3f}")
    for l in launches:
        print(f"{l['pos']:3d} L{l['level']} {l['role']:8s} {l['storage']:12s} {l['mode']:6s} {l['kernel'][:40]:40s} "
              f"alg {l['algorithmic_bytes'] / 1e6:8.2f} MB  hbm {l['hbm_bytes'] / 1e6:8.2f} MB  x{l['ratio']:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:6])
