"""Summarise a rocprofv3 kernel trace of bench.py: per-kernel/per-grid averages
of the V-cycle kernels and the in-cycle gaps.

  python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [--cycles N]

V-cycle dispatches are recognised as the repeating tail of the trace that
starts with the first fine-level smoothing kernel (k_mul2 on the fine level).
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("famg::", "")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel-prefix", default="spmv_stream_kernel")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # cycle kernels: everything after the last setup kernel (spgemm/sort/...)
    setup = ("spgemm", "row_sort", "k_t_", "sten", "k_diag", "scan", "narrow", "perm", "abs_row",
             "smooth_fix", "k_recip", "k_jacobi", "k_l2", "k_divs", "nn_step", "k_dot")
    last_setup = max(i for i, r in enumerate(rows) if any(s in r["Kernel_Name"] for s in setup))
    cyc = rows[last_setup + 1:]
    groups = collections.OrderedDict()
    for r in cyc:
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        groups.setdefault(key, []).append(d)
    total = sum(sum(v) for v in groups.values())
    print(f"{'kernel':34s} {'blocks':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'share':>6s}")
    for (k, g), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:34s} {g:9d} {len(v):6d} {sum(v)/len(v):9.2f} {min(v):9.2f} {100*sum(v)/total:5.1f}%")
    # gaps between consecutive dispatches inside the cycle region
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(cyc, cyc[1:])]
    gaps = [g for g in gaps if g < 50]
    if gaps:
        gaps.sort()
        print(f"kernel busy {total/1e3:.3f} ms over {len(cyc)} dispatches; median gap {gaps[len(gaps)//2]:.2f} us")


if __name__ == "__main__":
    main()
