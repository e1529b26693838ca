"""Run length (planes per workgroup) of the fused fine-level launches: both
launches timed on their own (amg_multigrid_fine_launch, 20 each, HIP events)
for flag fine_fuse = 1 (automatic: one round of workgroups) and fixed lengths."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)
N = 256
A = fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N)
mg = fa.sa_build_box(A, (N, N, N), (2, 2, 2), coarsest_dim=1000)
b = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, N ** 3), device="cuda:0")
z = torch.empty_like(b)
mg.apply(z, b)
torch.cuda.synchronize()
out = {}
for ff in (1, 4, 6, 8, 10, 12, 16, 20, 24, 32):
    fa.set_flag("fine_fuse", ff)
    for which in (0, 1):
        for _ in range(3):
            mg.fine_launch(which, z, b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            mg.fine_launch(which, z, b)
        e1.record(stream)
        e1.synchronize()
        out[f"ff{ff}_which{which}_us"] = round(1000 * e0.elapsed_time(e1) / 20, 2)
fa.set_flag("fine_fuse", 1)
print(json.dumps(out), flush=True)
