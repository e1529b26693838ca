"""Regression check for stale reads across kernels: builds the 64^3 SA
hierarchy (value codes off) N times and compares every R/P SpMV with scipy on
the downloaded CSR.  With physically contiguous allocations (the old
amg_set_alloc_policy(1) default) 12 of 12 builds gave a P_1 whose SELL copy held
half-smoothed values; with hipMalloc 0 of 12 (FAMG_CHECK_STORAGE=1 reports the
finalize-time check).  Usage: python scripts/alloc_coherence.py BUILDS MAX_LEVELS
"""
import sys, numpy as np, torch
sys.path[:0] = ["faer-amg_amd", "oracle"]
import faer_amg_amd as fa
ctx = fa.Context(0)
dims = (64, 64, 64)
fa.set_value_codes(False)
def dev(v): return torch.as_tensor(v, device="cuda:0")
def nbad(M):
    S = M.to_scipy()
    x = np.random.default_rng(1).standard_normal(S.shape[1])
    y = torch.empty(M.nrows, dtype=torch.float64, device="cuda:0")
    M.apply(y, dev(x)); ctx.synchronize(); y = y.cpu().numpy(); ref = S @ x
    return int(np.sum(np.abs(y - ref) > 1e-12 * np.abs(ref).max()))
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
for it in range(int(sys.argv[1])):
    mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100, max_levels=int(sys.argv[2]))
    out = [tuple(nbad(M) for M in mg.level(l)[::2] + (mg.level(l)[3],) if M is not None) for l in range(mg.levels())]
    print("build", it, out, flush=True)
    del mg
