"""Workload for rocprofv3 PMC passes over the C2 cycle (verdict r03 item 6).

Runs, on one GPU, in this order:
  * CAL: y = D x, D diagonal (n = 256^3) stored as DIA codes: one 4-B code word
    per row + x read + y written, exactly known bytes through the same DIA
    kernel family -- calibrates FETCH_SIZE (gfx950: half the bytes of 16-B/lane
    streams, MI355X_MICROARCH.md) for these kernels;
  * COPY: y.copy_(x) between k_trace_mark<<<3>>> and <<<4>>>: 8 n read, 8 n
    written by torch's vectorised copy (16 B/lane), the access width the
    guide's factor of 2 is stated for -- a second, independent calibration;
  * FINE: y = A_0 x (the bench's roofline kernel, DIA SET on the 7-pt 256^3);
  * k_trace_mark<<<1>>>, CYCLES eager V-cycles of the C2 hierarchy (the bench's),
    k_trace_mark<<<2>>>.
scripts/pmc_cycle_summary.py matches every dispatch between the marks to the
library's launch plan (written to gpurun_out/pmc_cycle_plan.json) and divides
the corrected HBM bytes by the plan's algorithmic bytes per launch.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

ITERS, CYCLES, N = 5, 5, 256
ctx = fa.Context(0)
n = N ** 3
D = fa.SparseMatOp.from_arrays(ctx, n, n, np.arange(n + 1, dtype=np.int64), np.arange(n, dtype=np.int64),
                               np.full(n, 2.0))
A = fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N)
mg = fa.sa_build_box(A, (N, N, N), (2, 2, 2), coarsest_dim=1000)
mg.set_graph(False)
x = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, n), device="cuda:0")
y = torch.empty_like(x)
z = torch.empty_like(x)
torch.cuda.synchronize()
mg.apply(z, x)  # workspaces, Jacobi codes
ctx.synchronize()
plan = mg.cycle_plan()
ctx.trace_mark(3)
for _ in range(ITERS):  # COPY: torch's vectorised copy, 16-B/lane streams (the guide's calibrated width)
    y.copy_(x)
ctx.synchronize()
ctx.trace_mark(4)
for _ in range(ITERS):
    D.apply(y, x)
ctx.synchronize()
assert torch.equal(y, 2.0 * x)
for _ in range(ITERS):
    A.apply(y, x)
ctx.synchronize()
ctx.trace_mark(1)
for _ in range(CYCLES):
    mg.apply(z, x)
ctx.trace_mark(2)
ctx.synchronize()
info = {"cal": D.spmv_info(), "fine": A.spmv_info(), "n": n, "iters": ITERS, "cycles": CYCLES}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(info, open(os.path.join(ROOT, "gpurun_out", "pmc_cycle_known.json"), "w"), indent=1)
json.dump(plan, open(os.path.join(ROOT, "gpurun_out", "pmc_cycle_plan.json"), "w"))
print(f"done: cal {info['cal']['kernel']} fine {info['fine']['kernel']} plan {len(plan)} launches")
