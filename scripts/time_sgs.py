"""Time one SGS step (sweep from e = 0, and the in-place step x <- x + S(b - A x))
on the 27-point 256^3 operator: fused plane-parity phases (three per step, four
per step) against the colour launches (ms per step, 20 reps), bitwise check.
Env switches FAMG_SGS27_TY / FAMG_SGS27_U / FAMG_SGS27_NW select the phase
kernel variant."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

n = int(os.environ.get("EDGE", "256"))
modes = [int(m) for m in os.environ.get("MODES", "1,2,0").split(",")]
ctx = fa.Context(0)
A = fa.SparseMatOp.aniso27(ctx, n, n, n, 1.0, 1.0, 0.01)
res = {}
for mode in modes:
    fa.set_sgs_fused(mode)
    S = fa.SymGaussSeidel(A)
    r = torch.as_tensor(np.random.default_rng(1).standard_normal(n ** 3), device="cuda:0")
    e = torch.empty_like(r)
    for _ in range(3):
        S.apply(e, r)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        S.apply(e, r)
    ctx.synchronize()
    res[mode] = ((time.perf_counter() - t0) / 20 * 1e3, e.cpu().numpy())
    del S
fa.set_sgs_fused(1)
tag = " ".join(f"{k}={os.environ.get(k)}" for k in ("FAMG_SGS27_TY", "FAMG_SGS27_U", "FAMG_SGS27_NW")
               if os.environ.get(k))
names = {0: "colour launches", 1: "three phases", 2: "four phases"}
base = res[modes[-1]][1]
print(f"[{tag or 'default'}] " + ", ".join(
    f"{names[m]} {res[m][0]:.3f} ms/step{'' if np.array_equal(res[m][1], base) else ' (NOT BITWISE)'}"
    for m in modes), flush=True)
