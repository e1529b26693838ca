"""ctypes front end of the C oracle (oracle/amg_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product.  PARITY UNPINNED (see
amg_oracle.h and DESIGN.md): the reference cannot be built here and has no
golden data, so this is a restatement cross-checked against np_oracle.py.

Besides thin wrappers this module holds the oracle's hierarchy driver, a
restatement of Hierarchy::coarsen (reference src/hierarchy.rs:190-248) with
box aggregates standing in for the modularity partitioner.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

i64 = C.c_int64
dbl = C.c_double
vp = C.c_void_p
P_I64 = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
P_DBL = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build():
    """Compile liboracle.so (gcc; part of __graft_entry__.build())."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        sig = {
            "orc_csr_import": (vp, [i64, i64, P_I64, P_I64, P_DBL]),
            "orc_csr_free": (None, [vp]),
            "orc_csr_dims": (None, [vp, P_I64]),
            "orc_csr_export": (None, [vp, P_I64, P_I64, P_DBL]),
            "orc_gen_laplace3d_7pt": (vp, [i64, i64, i64]),
            "orc_aniso27_stencil": (None, [dbl, dbl, dbl, P_DBL]),
            "orc_gen_aniso27": (vp, [i64, i64, i64, dbl, dbl, dbl]),
            "orc_gen_fd1d": (vp, [i64]),
            "orc_gen_laplace2d_5pt": (vp, [i64]),
            "orc_spmv": (None, [vp, P_DBL, P_DBL]),
            "orc_spmv_omp": (None, [vp, P_DBL, P_DBL]),
            "orc_diag_jacobi": (None, [vp, dbl, P_DBL]),
            "orc_diag_l1": (None, [vp, P_DBL]),
            "orc_diag_l2": (None, [vp, P_DBL]),
            "orc_greedy_coloring": (i64, [vp, P_I64]),
            "orc_sgs_apply_in_place": (None, [vp, P_I64, i64, P_DBL]),
            "orc_chol_factor": (C.c_int, [i64, P_DBL, P_DBL]),
            "orc_chol_solve": (None, [i64, P_DBL, P_DBL]),
            "orc_parspmm_new": (vp, [vp]),
            "orc_parspmm_apply": (None, [vp, P_DBL, P_DBL]),
            "orc_parspmm_free": (None, [vp]),
            "orc_spgemm": (vp, [vp, vp]),
            "orc_transpose": (vp, [vp]),
            "orc_smooth_interpolation": (vp, [vp, vp, dbl]),
            "orc_rap": (vp, [vp, vp, vp]),
            "orc_sa_tentative": (vp, [i64, P_I64, i64, P_DBL, P_DBL]),
            "orc_nn_stationary_l1": (None, [vp, i64, P_DBL]),
            "orc_box_aggregates": (i64, [i64, i64, i64, i64, i64, i64, P_I64, P_I64]),
            "orc_mg_new": (vp, [i64]),
            "orc_mg_free": (None, [vp]),
            "orc_mg_set_op": (None, [vp, i64, vp]),
            "orc_mg_set_transfer": (None, [vp, i64, vp, vp]),
            "orc_mg_set_diag": (None, [vp, i64, P_DBL]),
            "orc_mg_set_sgs": (None, [vp, i64, P_I64, i64]),
            "orc_mg_set_chol": (C.c_int, [vp, i64]),
            "orc_mg_set_csr_smoother": (None, [vp, i64, vp]),
            "orc_mg_set_cycle": (None, [vp, i64, i64]),
            "orc_mg_set_parallel": (None, [vp, i64, i64]),
            "orc_mg_apply": (None, [vp, P_DBL, P_DBL]),
            "orc_stationary_solve": (i64, [vp, vp, P_DBL, P_DBL, i64, dbl, P_DBL]),
            "orc_pcg_solve": (i64, [vp, vp, vp, P_DBL, P_DBL, i64, dbl, dbl, P_DBL]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class Csr:
    """Owned handle on an oracle CSR (usize indices, fp64 values)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("oracle returned a null CSR")
        self.h = handle

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_csr_free(self.h)
            self.h = None

    @classmethod
    def from_arrays(cls, nrows, ncols, rowptr, col, val):
        return cls(lib().orc_csr_import(int(nrows), int(ncols),
                                        np.ascontiguousarray(rowptr, np.int64),
                                        np.ascontiguousarray(col, np.int64),
                                        np.ascontiguousarray(val, np.float64)))

    @classmethod
    def from_scipy(cls, M):
        M = M.tocsr()
        M.sort_indices()
        return cls.from_arrays(M.shape[0], M.shape[1], M.indptr, M.indices, M.data)

    def dims(self):
        d = np.zeros(3, np.int64)
        lib().orc_csr_dims(self.h, d)
        return int(d[0]), int(d[1]), int(d[2])

    @property
    def nrows(self):
        return self.dims()[0]

    @property
    def ncols(self):
        return self.dims()[1]

    def arrays(self):
        m, n, nnz = self.dims()
        rp = np.zeros(m + 1, np.int64)
        ci = np.zeros(nnz, np.int64)
        va = np.zeros(nnz, np.float64)
        lib().orc_csr_export(self.h, rp, ci, va)
        return rp, ci, va

    def to_scipy(self):
        import scipy.sparse as sp
        m, n, _ = self.dims()
        rp, ci, va = self.arrays()
        return sp.csr_matrix((va, ci, rp), shape=(m, n))

    def spmv(self, x):
        y = np.empty(self.nrows, np.float64)
        lib().orc_spmv(self.h, np.ascontiguousarray(x, np.float64), y)
        return y


def laplace3d_7pt(nx, ny, nz):
    return Csr(lib().orc_gen_laplace3d_7pt(nx, ny, nz))


def aniso27(nx, ny, nz, ex=1.0, ey=1.0, ez=0.01):
    return Csr(lib().orc_gen_aniso27(nx, ny, nz, ex, ey, ez))


def aniso27_stencil(ex=1.0, ey=1.0, ez=0.01):
    c = np.zeros(27, np.float64)
    lib().orc_aniso27_stencil(ex, ey, ez, c)
    return c


def fd1d(n_elements):
    return Csr(lib().orc_gen_fd1d(n_elements))


def laplace2d_5pt(n_elements):
    return Csr(lib().orc_gen_laplace2d_5pt(n_elements))


def jacobi_diag(A, omega=0.66):
    d = np.empty(A.nrows)
    lib().orc_diag_jacobi(A.h, omega, d)
    return d


def l1_diag(A):
    d = np.empty(A.nrows)
    lib().orc_diag_l1(A.h, d)
    return d


def l2_diag(A):
    d = np.empty(A.nrows)
    lib().orc_diag_l2(A.h, d)
    return d


def greedy_coloring(A):
    c = np.zeros(A.nrows, np.int64)
    nc = lib().orc_greedy_coloring(A.h, c)
    return c, int(nc)


def sgs_apply(A, color, ncolors, r):
    r = np.array(r, np.float64, copy=True)
    lib().orc_sgs_apply_in_place(A.h, np.ascontiguousarray(color, np.int64), ncolors, r)
    return r


def spgemm(A, B):
    return Csr(lib().orc_spgemm(A.h, B.h))


def transpose(A):
    return Csr(lib().orc_transpose(A.h))


def smooth_interpolation(A, P, omega=0.66):
    return Csr(lib().orc_smooth_interpolation(A.h, P.h, omega))


def rap(R, A, P):
    return Csr(lib().orc_rap(R.h, A.h, P.h))


def sa_tentative(agg_of, naggs, nn):
    n = len(agg_of)
    cnn = np.zeros(naggs)
    P = Csr(lib().orc_sa_tentative(n, np.ascontiguousarray(agg_of, np.int64), naggs,
                                   np.ascontiguousarray(nn, np.float64), cnn))
    return P, cnn


def nn_stationary_l1(A, x, iters=3):
    x = np.array(x, np.float64, copy=True)
    lib().orc_nn_stationary_l1(A.h, iters, x)
    return x


def box_aggregates(dims, box):
    nx, ny, nz = dims
    agg = np.zeros(nx * ny * nz, np.int64)
    cd = np.zeros(3, np.int64)
    na = lib().orc_box_aggregates(nx, ny, nz, box[0], box[1], box[2], agg, cd)
    return agg, int(na), tuple(int(v) for v in cd)


class ParSpmm:
    """ParSpmmOp restatement (reference src/par_spmm.rs)."""

    def __init__(self, A):
        self.A = A
        self.h = lib().orc_parspmm_new(A.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_parspmm_free(self.h)

    def apply(self, x):
        y = np.empty(self.A.nrows)
        lib().orc_parspmm_apply(self.h, np.ascontiguousarray(x, np.float64), y)
        return y


class Multigrid:
    """Restatement of reference Multigrid (src/preconditioners/multigrid.rs:171-424).

    levels: list of dicts with keys A (Csr), smoother ('jacobi', 'l1', 'sgs',
    'chol', ('diag', array) or ('csr', Csr) -- an explicit smoother matrix such as
    BlockSmoother::into_sparse_mat), omega, and for every non-coarsest level R, P.
    """

    def __init__(self, levels, mu=1, steps=1, omega=0.66):
        L = lib()
        self.levels = levels  # keep CSR handles alive
        self.h = L.orc_mg_new(len(levels))
        for l, lev in enumerate(levels):
            A = lev["A"]
            L.orc_mg_set_op(self.h, l, A.h)
            if l + 1 < len(levels):
                L.orc_mg_set_transfer(self.h, l, lev["R"].h, lev["P"].h)
            sm = lev.get("smoother", "jacobi")
            if isinstance(sm, tuple) and sm[0] == "diag":
                L.orc_mg_set_diag(self.h, l, np.ascontiguousarray(sm[1], np.float64))
            elif sm == "jacobi":
                L.orc_mg_set_diag(self.h, l, jacobi_diag(A, lev.get("omega", omega)))
            elif sm == "l1":
                L.orc_mg_set_diag(self.h, l, l1_diag(A))
            elif sm == "l2":
                L.orc_mg_set_diag(self.h, l, l2_diag(A))
            elif sm == "sgs":
                color, nc = lev.get("coloring") or greedy_coloring(A)
                L.orc_mg_set_sgs(self.h, l, np.ascontiguousarray(color, np.int64), nc)
            elif isinstance(sm, tuple) and sm[0] == "csr":
                L.orc_mg_set_csr_smoother(self.h, l, sm[1].h)  # sm[1]: Csr kept alive by self.levels
            elif sm == "chol":
                if L.orc_mg_set_chol(self.h, l) != 0:
                    raise ValueError("coarse matrix is not SPD")
            else:
                raise ValueError(f"unknown smoother {sm!r}")
        L.orc_mg_set_cycle(self.h, mu, steps)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_mg_free(self.h)

    def set_parallel(self, nthreads):
        lib().orc_mg_set_parallel(self.h, 1, int(nthreads))

    def apply(self, rhs):
        out = np.empty(len(rhs))
        lib().orc_mg_apply(self.h, np.ascontiguousarray(rhs, np.float64), out)
        return out


def stationary_solve(A, mg, b, x0=None, max_iter=100, rel_tol=1e-8):
    x = np.zeros(A.nrows) if x0 is None else np.array(x0, np.float64, copy=True)
    hist = np.zeros(max_iter)
    it = lib().orc_stationary_solve(A.h, mg.h, np.ascontiguousarray(b, np.float64), x,
                                    max_iter, rel_tol, hist)
    return x, int(it), hist[:it]


def pcg_solve(A, b, mg=None, diag=None, x0=None, max_iter=1000, rel_tol=1e-8, abs_tol=0.0):
    x = np.zeros(A.nrows) if x0 is None else np.array(x0, np.float64, copy=True)
    hist = np.zeros(max_iter + 1)
    dptr = None if diag is None else np.ascontiguousarray(diag, np.float64).ctypes.data_as(C.c_void_p)
    it = lib().orc_pcg_solve(A.h, None if mg is None else mg.h, dptr,
                             np.ascontiguousarray(b, np.float64), x, max_iter, rel_tol,
                             abs_tol, hist)
    return x, int(it), hist[:min(it, max_iter)]


def composite_apply(A, components, rhs):
    """Composite::implementation (preconditioners/composite.rs:66-83): out = 0,
    ws = rhs; for c in c_{m-1}..c_0 then c_1..c_{m-1}: ws = c(ws) (apply_in_place),
    out += ws, ws = rhs - A out.  components: callables r -> c(r)."""
    rhs = np.ascontiguousarray(rhs, np.float64)
    out = np.zeros_like(rhs)
    ws = rhs.copy()
    m = len(components)
    for k in list(range(m - 1, -1, -1)) + list(range(1, m)):
        ws = components[k](ws)
        out = out + ws
        ws = rhs - A.spmv(out)
    return out


def sa_hierarchy_box(A, dims, box=(2, 2, 2), coarsest_dim=1000, max_levels=None,
                     omega=0.66, nn_iters=3, nn=None):
    """Hierarchy::coarsen restated (hierarchy.rs:190-248) for structured grids.

    Per level: box aggregates; tentative P (interpolation/mod.rs:754-805);
    one Jacobi smoothing step of P (:812-818, :927-946); R = P^T (:824-827);
    A_c = R (A P) (:828); coarse candidate post-processed by a 3-step L1
    StationaryIteration + thin QR (hierarchy.rs:219-228).
    Returns a list of level dicts {A, R, P, dims, nn}.
    """
    levels = []
    cur, cur_dims = A, tuple(dims)
    cur_nn = np.ones(cur.nrows) if nn is None else np.asarray(nn, np.float64)
    max_levels = max_levels or 10**9
    level = 1
    coarse_dim = None  # usize::MAX in the reference: always coarsen at least once
    while (coarse_dim is None or coarse_dim > coarsest_dim) and level < max_levels:
        agg, na, cdims = box_aggregates(cur_dims, box)
        Pt, cnn = sa_tentative(agg, na, cur_nn)
        P = smooth_interpolation(cur, Pt, omega)
        R = transpose(P)
        Ac = rap(R, cur, P)
        levels.append({"A": cur, "R": R, "P": P, "dims": cur_dims, "nn": cur_nn})
        cnn = nn_stationary_l1(Ac, cnn, nn_iters)
        cur, cur_dims, cur_nn = Ac, cdims, cnn
        coarse_dim = cur.nrows
        level += 1
    levels.append({"A": cur, "dims": cur_dims, "nn": cur_nn})
    return levels
