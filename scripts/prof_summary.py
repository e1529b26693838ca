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


CYCLE_HELPERS = ("k_mul2", "k_mul2_coded", "k_gemv", "k_gather_idx")


def setup_kernel(name):
    """Setup kernels (value tables, storage fills, SpGEMM) that a trace of ~23
    builds can count as often as the cycles: all k_* but the cycle's helpers."""
    s = short(name)
    return s.startswith("k_") and s not in CYCLE_HELPERS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--cycles", type=int, default=23, help="V-cycles in the trace (warm-up + timed)")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # cycle kernels: the (kernel, grid) pairs dispatched once per V-cycle, i.e.
    # at least --cycles times (warm-up + timed cycles of bench.py)
    count = collections.Counter((r["Kernel_Name"], r["Grid_Size_X"]) for r in rows)
    cyc = [r for r in rows if args.cycles <= count[(r["Kernel_Name"], r["Grid_Size_X"])] <= args.cycles + 2
           and not r["Kernel_Name"].startswith("__amd") and not setup_kernel(r["Kernel_Name"])]
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
    per_cycle = total / args.cycles
    print(f"per V-cycle: {per_cycle / 1e3:.3f} ms of kernel time (sum of the kernels above / {args.cycles})")
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(cyc, cyc[1:])]
    gaps = [g for g in gaps if g < 50]
    if gaps:
        gaps.sort()
        print(f"kernel busy {total/1e3:.3f} ms over {len(cyc)} dispatches; median gap {gaps[len(gaps)//2]:.2f} us")


if __name__ == "__main__":
    main()
