"""Fine-SpMV HBM traffic from the rocprofv3 PMC passes of scripts/pmc_fine_spmv.py.

  python scripts/pmc_summary.py FETCH.csv WRITE.csv KNOWN.json OUT.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  The first ITERS SELL
dispatches are the calibration (diagonal matrix, n = 256^3: exactly the matrix
stream bytes recorded in KNOWN.json + 8 n read, 8 n written); the last ITERS
are the 7-point operator.  Read bytes = FETCH_SIZE * 1024 * (known calibration bytes /
calibration FETCH_SIZE bytes) -- on gfx950 that factor is ~2 for streaming
loads (MI355X_MICROARCH.md, HBM section).
"""
import csv
import json
import statistics
import sys

ITERS = 10
N = 256 ** 3


def sell_values(path, counter, kernel="spmv_sell_kernel"):
    rows = [r for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    vals = [float(r["Counter_Value"]) * 1024.0 for r in rows]
    assert len(vals) == 2 * ITERS, (path, len(vals))
    return vals[:ITERS], vals[ITERS:]


def main(fetch_csv, write_csv, known_json, out_json):
    global N
    known = json.load(open(known_json))
    N = known.get("n", N)
    kern = known.get("kernel", "spmv_%s_kernel" % known["fine"]["kernel"])
    assert known["cal"]["kernel"] == known["fine"]["kernel"], known
    cal_f, fine_f = sell_values(fetch_csv, "FETCH_SIZE", kern)
    cal_w, fine_w = sell_values(write_csv, "WRITE_SIZE", kern)
    cal_read_known = known["cal"]["stream_bytes"] + 8 * N
    factor = cal_read_known / statistics.median(cal_f)
    read = statistics.median(fine_f) * factor
    write = statistics.median(fine_w)
    out = {
        "kernel": kern + "<SET> on " + known.get("workload", "A_0 (7-pt 256^3)"),
        "storage": known["fine"],
        "algorithmic_bytes_per_launch": known["fine"]["stream_bytes"] + 16 * N,
        "fetch_correction_factor": round(factor, 4),
        "calibration": {"known_read_bytes": cal_read_known,
                        "fetch_size_bytes": statistics.median(cal_f),
                        "write_size_bytes": statistics.median(cal_w), "known_write_bytes": 8 * N},
        "read_bytes_per_launch": round(read),
        "write_bytes_per_launch": round(write),
        "hbm_bytes_per_launch": round(read + write),
    }
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
