"""Summarise a rocprofv3 kernel trace of bench.py: the timed V-cycles only,
per kernel, per V-cycle, and (with --plan) per launch of the library's own
launch plan with its algorithmic bytes and achieved GB/s.

  python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps K [--plan plan.json]

bench.py brackets its K timed V-cycles with k_trace_mark<<<1>>> and
k_trace_mark<<<2>>> (amg_trace_mark); every dispatch between the two marks is
one of the K cycles' launches, whatever kernel it is and however many times a
cycle launches it (SGS colour sweeps run ~30 times per cycle).  The summary
therefore sums to the timed cycle's kernel time.  --plan (bench.py --plan-out)
is the ordered launch list of one cycle (amg_multigrid_cycle_plan); dispatches
are matched to it position by position within each cycle.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("famg::", "")
    return name


def timed_region(rows):
    """Dispatches between the k_trace_mark<<<1>>> and <<<2>>> marks."""
    marks = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith("k_trace_mark")]
    begin = end = None
    for i in marks:
        blocks = int(rows[i]["Grid_Size_X"]) // int(rows[i]["Workgroup_Size_X"])
        if blocks == 1:
            begin = i
        elif blocks == 2 and begin is not None:
            end = i
            break
    if begin is None or end is None:
        raise SystemExit("no k_trace_mark pair in the trace (bench.py marks its timed cycles)")
    return rows[begin + 1:end]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="timed V-cycles (bench.py --steps)")
    ap.add_argument("--plan", default=None, help="bench.py --plan-out JSON (launch plan of one cycle)")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cyc = timed_region(rows)
    K = args.steps
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in cyc]
    groups = collections.OrderedDict()
    for r, d in zip(cyc, dur):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        groups.setdefault(key, []).append(d)
    total = sum(dur)
    print(f"timed region: {len(cyc)} dispatches over {K} V-cycles = {len(cyc) / K:.2f} per cycle")
    print(f"{'kernel':44s} {'blocks':>7s} {'/cycle':>6s} {'avg_us':>8s} {'min_us':>8s} {'us/cycle':>9s} {'share':>6s}")
    for (k, g), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:44s} {g:7d} {len(v) / K:6.2f} {sum(v) / len(v):8.2f} {min(v):8.2f} "
              f"{sum(v) / K:9.2f} {100 * sum(v) / total:5.1f}%")
    first = int(cyc[0]["Start_Timestamp"])
    last = int(cyc[-1]["End_Timestamp"])
    print(f"per V-cycle: {total / K / 1e3:.4f} ms of kernel time (all dispatches between the marks / {K}); "
          f"span {(last - first) / K / 1e6:.4f} ms per cycle incl. gaps")
    if not args.plan:
        return
    plan = json.load(open(args.plan))["plan"]
    L = len(plan)
    if len(cyc) != K * L:
        print(f"plan has {L} launches per cycle but the region holds {len(cyc)} = {len(cyc) / K:.2f} x {K}: "
              "per-launch join skipped")
        return
    print(f"\nper launch (plan order; {L} launches, times = mean over {K} cycles):")
    print(f"{'#':>3s} {'lvl':>3s} {'role':8s} {'storage':12s} {'mode':6s} {'kernel':44s} {'us':>8s} "
          f"{'MB':>9s} {'GB/s':>7s}")
    tot_b = 0
    for j, p in enumerate(plan):
        ts = [dur[c * L + j] for c in range(K)]
        t = sum(ts) / K
        tot_b += p["bytes"]
        print(f"{j:3d} {p['level']:3d} {p['role']:8s} {p['name']:12s} {p['mode']:6s} "
              f"{short(cyc[j]['Kernel_Name'])[:44]:44s} {t:8.2f} {p['bytes'] / 1e6:9.2f} "
              f"{p['bytes'] / (t * 1e3) if t > 0 else 0:7.0f}")
    print(f"plan bytes per cycle {tot_b / 1e9:.4f} GB over {total / K / 1e3:.4f} ms of kernel time = "
          f"{tot_b / (total / K * 1e3):.0f} GB/s")


if __name__ == "__main__":
    main()
