"""Times the fused fine-level launches on their own (amg_multigrid_fine_launch),
20 launches each, HIP events on the library stream; prints one JSON line.
FAMG_FINE_DBG (read per launch) switches parts off for timing experiments."""
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
for dbg in sys.argv[1:] or ["0"]:
    os.environ["FAMG_FINE_DBG"] = dbg
    for which in (0, 1):
        for _ in range(3):
            mg.fine_launch(which, z, b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            mg.fine_launch(which, z, b)
        e1.record(stream)
        e1.synchronize()
        out[f"dbg{dbg}_which{which}_us"] = round(1000 * e0.elapsed_time(e1) / 20, 2)
os.environ["FAMG_FINE_DBG"] = "0"
print(json.dumps(out), flush=True)
