"""Each fused grid transfer (fuse.hip) of a box hierarchy's fine level against the
oracle's row sums of the unfused steps: mismatch counts and the first mismatching
grid points (debugging aid; the parity test is test_fused_grid_transfers_*)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import faer_amg_amd as fa  # noqa: E402
import oracle as O  # noqa: E402

dims = tuple(int(v) for v in os.environ.get("DIMS", "64,48,40").split(","))
ctx = fa.Context(0)
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
A0, S0, R0, P0 = mg.level(0)
OA = O.Csr.from_arrays(*A0.dims(), *A0.arrays())
OR = O.Csr.from_arrays(*R0.dims(), *R0.arrays())
OP = O.Csr.from_arrays(*P0.dims(), *P0.arrays())
n, nc = A0.nrows, R0.nrows
T = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float64), device="cuda:0")  # noqa: E731
ones = T(np.ones(n))
dd = torch.empty_like(ones)
S0.apply(dd, ones)
ctx.synchronize()
d = dd.cpu().numpy()
rng = np.random.default_rng(3)
f, x, vc = rng.standard_normal(n), rng.standard_normal(n), rng.standard_normal(nc)
cdims = tuple(-(-v // 2) for v in dims)


def report(name, got, want, grid):
    bad = np.nonzero(got != want)[0]
    print(f"{name}: {len(bad)} of {len(want)} differ, max abs {np.max(np.abs(got - want)) if len(bad) else 0:.3e}")
    for i in bad[:8]:
        X, Y, Z = i % grid[0], (i // grid[0]) % grid[1], i // (grid[0] * grid[1])
        print(f"   ({X},{Y},{Z}) got {got[i]!r} want {want[i]!r}")


out = T(np.full(nc, np.nan))
for xm in ("fold", "x"):
    ok = mg.fused_transfer(0, "restrict", T(f), None, None if xm == "fold" else T(x), out)
    ctx.synchronize()
    xo = d * f if xm == "fold" else x
    want = OR.spmv(f - OA.spmv(xo))
    if ok:
        report(f"restrict[{xm}]", out.cpu().numpy(), want, cdims)
    else:
        print(f"restrict[{xm}]: not fused")
outf = T(np.full(n, np.nan))
for xm in ("fold", "x"):
    ok = mg.fused_transfer(0, "interp", T(vc), T(f), None if xm == "fold" else T(x), outf)
    ctx.synchronize()
    v = (d * f if xm == "fold" else x) + OP.spmv(vc)
    want = v + d * (f - OA.spmv(v))
    if ok:
        report(f"interp[{xm}]", outf.cpu().numpy(), want, dims)
    else:
        print(f"interp[{xm}]: not fused")
