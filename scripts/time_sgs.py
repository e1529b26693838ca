"""Time one SGS step (sweep from e = 0) on the 27-point 256^3 operator: the
fused plane-parity phases against the colour launches (ms per step, 20 reps).
Env switches FAMG_SGS27_TY / FAMG_SGS27_U select the phase kernel variant."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

n = int(os.environ.get("EDGE", "256"))
ctx = fa.Context(0)
A = fa.SparseMatOp.aniso27(ctx, n, n, n, 1.0, 1.0, 0.01)
res = {}
for fused in (True, False):
    fa.set_sgs_fused(fused)
    S = fa.SymGaussSeidel(A)
    r = torch.as_tensor(np.random.default_rng(1).standard_normal(n ** 3), device="cuda:0")
    e = torch.empty_like(r)
    for _ in range(3):
        S.apply(e, r)
    ctx.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    ctx.join_torch(False) if hasattr(ctx, "join_torch") else None
    import time
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        S.apply(e, r)
    ctx.synchronize()
    res[fused] = ((time.perf_counter() - t0) / 20 * 1e3, e.cpu().numpy())
    del S
fa.set_sgs_fused(True)
print(f"TY={os.environ.get('FAMG_SGS27_TY', '16')} U={os.environ.get('FAMG_SGS27_U', '1')}: "
      f"fused {res[True][0]:.3f} ms/step, colour launches {res[False][0]:.3f} ms/step, "
      f"bitwise {np.array_equal(res[True][1], res[False][1])}", flush=True)
