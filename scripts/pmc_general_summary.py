"""HBM traffic of the roofline.general SpMV from the PMC passes of scripts/pmc_general.py.

  python scripts/pmc_general_summary.py FETCH.csv WRITE.csv KNOWN.json OUT.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  The first ITERS dispatches of
the kernel are the calibration (known read bytes: the format's stream bytes +
8n of x; written 8n), the last ITERS the general operator.  Read bytes =
FETCH_SIZE * 1024 * (known calibration bytes / calibration FETCH_SIZE bytes), as
MI355X_MICROARCH.md's HBM section prescribes for a kernel's own access widths.
"""
import csv
import json
import statistics
import sys

ITERS = 10


def values(path, counter, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    vals = [float(r["Counter_Value"]) * 1024.0 for r in rows]
    assert len(vals) == 2 * ITERS, (path, len(vals))
    return vals[:ITERS], vals[ITERS:]


def main(fetch_csv, write_csv, known_json, out_json):
    known = json.load(open(known_json))
    n, nnz = known["n"], known["nnz"]
    kern = {"xsell": known.get("xs_kernel", "spmv_xs_burst_kernel"), "sell": "spmv_sell_kernel"}[known["gen"]["kernel"]]
    cal_f, gen_f = values(fetch_csv, "FETCH_SIZE", kern)
    cal_w, gen_w = values(write_csv, "WRITE_SIZE", kern)
    cal_read = known["cal"]["stream_bytes"] + 8 * n
    factor = cal_read / statistics.median(cal_f)
    read = statistics.median(gen_f) * factor
    write = statistics.median(gen_w)
    out = {
        "kernel": kern + "<SET> on the roofline.general operator (random 7-pt 256^3, window 4096)",
        "storage": known["gen"],
        "format_bytes_per_launch": known["gen"]["stream_bytes"] + 16 * n,
        "csr_bytes_per_launch": 12 * nnz + 4 * (n + 1) + 16 * n,
        "fetch_correction_factor": round(factor, 4),
        "calibration": {"known_read_bytes": cal_read, "fetch_size_bytes": statistics.median(cal_f),
                        "write_size_bytes": statistics.median(cal_w), "known_write_bytes": 8 * n},
        "read_bytes_per_launch": round(read),
        "write_bytes_per_launch": round(write),
        "hbm_bytes_per_launch": round(read + write),
    }
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
