"""Independent numpy/scipy restatement of the V-cycle path.

TEST INFRASTRUCTURE ONLY.  Written separately from amg_oracle.c (different
code, scipy's own SpMV/SpGEMM summation order) so that the two restatements
check each other; agreement is to rounding, not bitwise.  Cites the reference
lines it follows.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp


def laplace3d_7pt(nx, ny, nz):
    def t(n):
        return sp.diags([-np.ones(n - 1), np.zeros(n), -np.ones(n - 1)], [-1, 0, 1])
    ix, iy, iz = sp.identity(nx), sp.identity(ny), sp.identity(nz)
    A = (sp.kron(iz, sp.kron(iy, t(nx))) + sp.kron(iz, sp.kron(t(ny), ix))
         + sp.kron(t(nz), sp.kron(iy, ix)))
    A = A + 6.0 * sp.identity(nx * ny * nz)
    A = A.tocsr()
    A.sort_indices()
    return A


def aniso27(nx, ny, nz, ex=1.0, ey=1.0, ez=0.01):
    """eps_x T(x) M M + eps_y M T(y) M + eps_z M M T(z); x fastest index."""
    def T(n):
        return sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1])

    def M(n):
        return sp.diags([np.ones(n - 1) / 6, 4 * np.ones(n) / 6, np.ones(n - 1) / 6], [-1, 0, 1])
    A = (ex * sp.kron(M(nz), sp.kron(M(ny), T(nx))) + ey * sp.kron(M(nz), sp.kron(T(ny), M(nx)))
         + ez * sp.kron(T(nz), sp.kron(M(ny), M(nx))))
    A = A.tocsr()
    A.sort_indices()
    return A


def fd1d(n_elements):
    """examples/simple_geometric.rs:96-113."""
    h = 1.0 / n_elements
    n = n_elements - 1
    return sp.diags([-np.ones(n - 1) / h**2, 2 * np.ones(n) / h**2, -np.ones(n - 1) / h**2],
                    [-1, 0, 1]).tocsr()


def interp1d(n_coarse):
    """make_interpolation (simple_geometric.rs:62-75)."""
    n_fine = 2 * n_coarse + 1
    rows, cols, vals = [], [], []
    for c in range(n_coarse):
        for off, v in ((0, 0.5), (1, 1.0), (2, 0.5)):
            rows.append(2 * c + off); cols.append(c); vals.append(v)
    return sp.csr_matrix((vals, (rows, cols)), shape=(n_fine, n_coarse))


def restrict1d(n_coarse):
    """make_restriction (simple_geometric.rs:80-93): full weighting = P^T / 2."""
    n_fine = 2 * n_coarse + 1
    rows, cols, vals = [], [], []
    for c in range(n_coarse):
        for off, v in ((0, 0.25), (1, 0.5), (2, 0.25)):
            rows.append(c); cols.append(2 * c + off); vals.append(v)
    return sp.csr_matrix((vals, (rows, cols)), shape=(n_coarse, n_fine))


def laplace2d_5pt(n_elements):
    h = 1.0 / n_elements
    m = n_elements - 1
    t = sp.diags([-np.ones(m - 1), 2 * np.ones(m), -np.ones(m - 1)], [-1, 0, 1])
    A = (sp.kron(sp.identity(m), t) + sp.kron(t, sp.identity(m))) / h**2
    A = A.tocsr()
    A.sort_indices()
    return A


def gmg2d_levels(n_elements, coarsest_elements):
    """Config C1: 2-D restatement of simple_geometric main (:200-224): rediscretized
    coarse operators, P = kron(P1,P1), R = kron(R1,R1), Jacobi 0.66, Cholesky coarsest."""
    levels = []
    ne = n_elements
    while True:
        A = laplace2d_5pt(ne)
        lev = {"A": A}
        levels.append(lev)
        if ne <= coarsest_elements:
            break
        nc = ne // 2 - 1
        P1, R1 = interp1d(nc), restrict1d(nc)
        lev["P"] = sp.kron(P1, P1).tocsr()
        lev["R"] = sp.kron(R1, R1).tocsr()
        for M in (lev["P"], lev["R"]):
            M.sort_indices()
        ne //= 2
    return levels


def gmg1d_levels(n_elements, refinement, base_elements=10):
    """examples/simple_geometric.rs:200-224 (1-D, `refinement` coarse levels)."""
    levels = [{"A": fd1d(n_elements)}]
    for level in range(1, refinement + 1):
        ce = base_elements * 2 ** (refinement - level)
        cd = ce - 1
        levels[-1]["R"] = restrict1d(cd)
        levels[-1]["P"] = interp1d(cd)
        levels.append({"A": fd1d(ce)})
    return levels


class Multigrid:
    """multigrid.rs:251-424 with numpy vectors. Smoothers: 'jacobi' (omega/a_ii),
    'l1', 'sgs' (greedy coloring), 'chol' (dense Cholesky)."""

    def __init__(self, levels, mu=1, steps=1, omega=0.66):
        self.levels, self.mu, self.steps = levels, mu, steps
        self.sm = []
        for lev in levels:
            A = lev["A"].tocsr()
            kind = lev.get("smoother", "jacobi")
            d = A.diagonal()
            if callable(kind):                      # any Precond r -> M r
                self.sm.append(("fn", kind))
            elif kind == "jacobi":
                self.sm.append(("diag", omega / d))
            elif kind == "l1":
                self.sm.append(("diag", 1.0 / np.asarray(abs(A).sum(axis=1)).ravel()))
            elif kind == "sgs":
                color, nc = greedy_coloring(A)
                self.sm.append(("sgs", (color, nc, 1.0 / d)))
            elif kind == "chol":
                self.sm.append(("chol", sla.cho_factor(A.toarray(), lower=True)))
            else:
                raise ValueError(kind)

    def _pc(self, l, r):
        kind, data = self.sm[l]
        if kind == "fn":
            return data(r)
        if kind == "diag":
            return data * r
        if kind == "chol":
            return sla.cho_solve(data, r)
        color, nc, dinv = data
        return sgs(self.levels[l]["A"], color, nc, dinv, r)

    def _smooth(self, l, x, b):
        A = self.levels[l]["A"]
        for _ in range(self.steps):
            r = b - A @ x
            x = x + self._pc(l, r)
        return x

    def _cycle(self, v, f, l):
        if l == len(self.levels) - 1:
            return self._pc(l, f)
        A, R, P = self.levels[l]["A"], self.levels[l]["R"], self.levels[l]["P"]
        v = self._smooth(l, v, f)
        fc = R @ (f - A @ v)
        vc = np.zeros(R.shape[0])
        for _ in range(self.mu):
            vc = self._cycle(vc, fc, l + 1)
        v = v + P @ vc
        return self._smooth(l, v, f)

    def apply(self, rhs):
        return self._cycle(np.zeros(len(rhs)), np.asarray(rhs, np.float64), 0)


def greedy_coloring(A):
    A = A.tocsr()
    n = A.shape[0]
    color = np.zeros(n, np.int64)
    for i in range(n):
        nb = A.indices[A.indptr[i]:A.indptr[i + 1]]
        used = set(color[nb[nb < i]].tolist())
        c = 0
        while c in used:
            c += 1
        color[i] = c
    return color, int(color.max()) + 1 if n else 0


def sgs(A, color, nc, dinv, r):
    """Multicolor SGS from e = 0 (forward 0..C-1, backward C-2..0)."""
    A = A.tocsr()
    e = np.zeros(len(r))
    order = list(range(nc)) + list(range(nc - 2, -1, -1))
    for c in order:
        rows = np.nonzero(color == c)[0]
        Ae = A[rows] @ e
        e[rows] = e[rows] + dinv[rows] * (r[rows] - Ae)
    return e


def stationary(A, M, b, max_iter, tol):
    """simple_geometric.rs:117-158."""
    x = np.zeros(len(b))
    bn = np.linalg.norm(b)
    hist = []
    while True:
        r = b - A @ x
        rel = np.linalg.norm(r) / bn
        hist.append(rel)
        if rel < tol or len(hist) >= max_iter:
            break
        x = x + M(r)
    return x, hist


def pcg(A, b, M, max_iter, tol):
    x = np.zeros(len(b))
    r = b.copy()
    bn = np.linalg.norm(b)
    z = M(r)
    p = z.copy()
    rz = r @ z
    for it in range(1, max_iter + 1):
        Ap = A @ p
        alpha = rz / (p @ Ap)
        x = x + alpha * p
        r = r - alpha * Ap
        if np.linalg.norm(r) <= tol * bn:
            return x, it
        z = M(r)
        rzn = r @ z
        p = z + (rzn / rz) * p
        rz = rzn
    return x, max_iter + 1


def box_aggregates(dims, box):
    nx, ny, nz = dims
    bx, by, bz = box
    cx, cy, cz = -(-nx // bx), -(-ny // by), -(-nz // bz)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    agg = (x // bx + cx * (y // by + cy * (z // bz))).ravel()
    return agg.astype(np.int64), cx * cy * cz, (cx, cy, cz)


def sa_level(A, agg, naggs, nn, omega=0.66):
    """interpolation/mod.rs:754-836 for one candidate, block size 1."""
    A = A.tocsr()
    n = A.shape[0]
    norms = np.sqrt(np.bincount(agg, weights=nn * nn, minlength=naggs))
    Pt = sp.csr_matrix((nn / norms[agg], (np.arange(n), agg)), shape=(n, naggs))
    Dinv = sp.diags(omega / A.diagonal())
    P = (Pt - Dinv @ (A @ Pt)).tocsr()
    R = P.T.tocsr()
    Ac = (R @ (A @ P)).tocsr()
    for M in (P, R, Ac):
        M.sort_indices()
    return P, R, Ac, norms


def nn_stationary_l1(A, x, iters=3):
    """hierarchy.rs:219-228 with smoothers.rs:146-158 (r = x - A x quirk) + QR."""
    d = 1.0 / np.asarray(abs(A).sum(axis=1)).ravel()
    x = d * x
    for _ in range(1, iters):
        x = x + d * (x - A @ x)
    return x / np.linalg.norm(x)


def sa_hierarchy_box(A, dims, box=(2, 2, 2), coarsest_dim=1000, omega=0.66):
    levels = []
    cur, cur_dims, nn = A.tocsr(), tuple(dims), np.ones(A.shape[0])
    coarse_dim = None
    while coarse_dim is None or coarse_dim > coarsest_dim:
        agg, na, cdims = box_aggregates(cur_dims, box)
        P, R, Ac, cnn = sa_level(cur, agg, na, nn, omega)
        levels.append({"A": cur, "P": P, "R": R, "dims": cur_dims})
        nn = nn_stationary_l1(Ac, cnn)
        cur, cur_dims = Ac, cdims
        coarse_dim = Ac.shape[0]
    levels.append({"A": cur, "dims": cur_dims})
    return levels


# ------------------------------------------------------------- dataset loaders

def load_mtx(path):
    """Matrix Market coordinate file -> scipy CSR, restating the reference's
    load_matrix_triplets (utils.rs:508-534: 0.0 entries dropped, symmetric
    entries mirrored) on top of the matrix-market-rs 0.1.3 parser (1-based
    indices, real/integer/pattern fields) and faer's try_new_from_triplets
    (duplicates summed in file order, sorted columns).  Pure-Python parsing,
    independent of the library's mmap/strtod parser."""
    with open(path) as f:
        lines = f.read().split("\n")
    head = lines[0].lower().split()
    assert head[0] == "%%matrixmarket" and head[2] == "coordinate"
    field, sym = head[3], head[4]
    k = 1
    while lines[k].strip() == "" or lines[k].lstrip().startswith("%"):
        k += 1
    m, n, nnz = (int(t) for t in lines[k].split())
    trip = []
    count = 0
    for line in lines[k + 1:]:
        s = line.strip()
        if not s or s.startswith("%"):
            continue
        t = s.split()
        count += 1
        i, j = int(t[0]) - 1, int(t[1]) - 1
        v = 1.0 if field == "pattern" else float(t[2])
        if v == 0.0:
            continue
        trip.append((i, j, v))
        if sym == "symmetric" and i != j:
            trip.append((j, i, v))
    assert count == nnz
    return triplets_to_csr(m, n, trip)


def triplets_to_csr(m, n, trip):
    rows = [dict() for _ in range(m)]
    for i, j, v in trip:  # file order: duplicates summed left to right
        rows[i][j] = rows[i][j] + v if j in rows[i] else v
    rp, ci, va = [0], [], []
    for r in rows:
        for j in sorted(r):
            ci.append(j)
            va.append(r[j])
        rp.append(len(ci))
    return sp.csr_matrix((np.asarray(va, float), np.asarray(ci, np.int64), np.asarray(rp, np.int64)),
                         shape=(m, n))


def load_mfem(directory, name, delete_boundary=True):
    """load_mfem_linear_system (utils.rs:269-350) without the VTK mesh:
    returns (A, rhs (n x k), coords (n x d), boundary (sorted unique),
    solution_to_mesh, mesh_to_solution (-1 = deleted))."""
    import os
    base = os.path.join(directory, name)
    with open(base + ".bdy") as f:
        bl = f.read().split("\n")
    expect = int(bl[0].strip())
    bidx = [int(s) for s in (x.strip() for x in bl[1:]) if s]   # utils.rs:364-395
    assert len(bidx) == expect
    boundary = sorted(set(bidx))
    A = load_mtx(base + ".mtx")
    n = A.shape[0]
    assert A.shape[0] == A.shape[1]
    with open(base + ".coords") as f:                            # utils.rs:397-415
        coords = [[float(t) for t in line.split()] for line in f if line.split()]
    assert len(coords) == n
    with open(base + ".rhs") as f:                               # utils.rs:417-430
        flat = [float(t) for t in f.read().split()]
    assert len(flat) % n == 0
    k = len(flat) // n
    rhs_full = np.asarray(flat).reshape(k, n).T                 # column-major (utils.rs:308-315)
    if delete_boundary:                                         # utils.rs:446-480
        isb = np.zeros(n, bool)
        isb[boundary] = True
        sel = np.flatnonzero(~isb)
    else:
        sel = np.arange(n)
    m2s = -np.ones(n, np.int64)
    m2s[sel] = np.arange(len(sel))
    if delete_boundary:
        # filter the (already summed) matrix: same as filtering the triplets,
        # since rows/columns are removed whole
        A = A[sel][:, sel].tocsr()
        A.sort_indices()
    C = np.asarray([coords[i] for i in sel]) if len(sel) else np.zeros((0, 0))
    return A, rhs_full[sel], C, np.asarray(boundary, np.int64), sel.astype(np.int64), m2s


# ------------------------------------------------------------ block smoother

def block_smoother(A, node_partition, block_size=1):
    """BlockSmoother with BlockSolver(Cholesky) blocks (block_smoothers.rs:80-291):
    returns r -> M r.  Blocks: aggregates' nodes ascending (BTreeSet order),
    diagonally compensated (diagonally_compensate :293-324 for block_size 1:
    a_ii += 0.5 sqrt(a_ii/a_jj) |a_ij| per coupling leaving the aggregate;
    diagonally_compensate_vector :326-400: node diagonal blocks += 0.5 U S U^T
    of the SVD of -A_IJ per coupled outside node J), each solved with a dense
    Cholesky (scipy cho_solve)."""
    A = A.tocsr()
    v = int(block_size)
    part = np.asarray(node_partition, np.int64)
    nagg = int(part.max()) + 1 if len(part) else 0
    d = A.diagonal()
    blocks = []
    for a in range(nagg):
        nodes = np.flatnonzero(part == a)
        if len(nodes) == 0:
            continue
        idx = (nodes[:, None] * v + np.arange(v)[None, :]).ravel()
        pos = {int(g): k for k, g in enumerate(nodes)}
        B = np.zeros((len(idx), len(idx)))
        for k, I in enumerate(nodes):
            outside = set()
            for oi in range(v):
                i = I * v + oi
                for e in range(A.indptr[i], A.indptr[i + 1]):
                    j = int(A.indices[e])
                    J, oj = j // v, j % v
                    if J in pos:
                        B[k * v + oi, pos[J] * v + oj] += A.data[e]
                    elif v == 1:
                        B[k, k] += 0.5 * np.sqrt(d[i] / d[j]) * abs(A.data[e])
                    else:
                        outside.add(J)
            for J in sorted(outside):
                M = -A[I * v:(I + 1) * v, J * v:(J + 1) * v].toarray()
                U, S, _ = np.linalg.svd(M)
                B[k * v:(k + 1) * v, k * v:(k + 1) * v] += 0.5 * (U * S) @ U.T
        blocks.append((idx, sla.cho_factor(B, lower=True)))

    def apply(r):
        out = np.zeros(len(r))
        for idx, f in blocks:
            out[idx] = sla.cho_solve(f, r[idx])
        return out
    return apply
