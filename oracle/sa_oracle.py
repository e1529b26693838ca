"""Pure-Python / numpy restatement of the general smoothed-aggregation setup
(config C5) -- TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of
faer-amg_amd/csrc/sa.hip and gen.cpp, never by the product.

PARITY UNPINNED: the reference is Rust with a non-vendored faer
fork and cannot be built here; it ships no fixtures.  Each function restates the
reference item it cites (paths relative to the reference root) with the
determinism rules DESIGN.md 10 fixes where the reference leaves the order to
unstable sorts (strength ties by column, MIS degree ties by node index).  The
strength graph and aggregation are restated operation for operation (same
summation order), so they compare bitwise; the SVD / eigen / QR steps use
LAPACK (numpy), an independent algorithm, and compare to rounding.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp


# ------------------------------------------------------------------ generator

def _splitmix64(z):
    M = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def _unit(seed, i):
    M = (1 << 64) - 1
    return float(_splitmix64((seed + i * 0x9E3779B97F4A7C15) & M) >> 11) * 2.0 ** -53


def q1_reference_stiffness(nu):
    """24 x 24 trilinear-hex stiffness of the unit cube, E = 1 (2x2x2 Gauss)."""
    lam = nu / ((1 + nu) * (1 - 2 * nu))
    mu = 1 / (2 * (1 + nu))
    D = np.zeros((6, 6))
    D[:3, :3] = lam
    D[np.arange(3), np.arange(3)] += 2 * mu
    D[3:, 3:] = np.eye(3) * mu
    K = np.zeros((24, 24))
    g = 1 / math.sqrt(3)
    for gz in (0, 1):
        for gy in (0, 1):
            for gx in (0, 1):
                xi, et, ze = (g if gx else -g), (g if gy else -g), (g if gz else -g)
                B = np.zeros((6, 24))
                for a in range(8):
                    sa, ta, ua = (1 if a & 1 else -1), (1 if a & 2 else -1), (1 if a & 4 else -1)
                    dx = 0.25 * sa * (1 + et * ta) * (1 + ze * ua)
                    dy = 0.25 * ta * (1 + xi * sa) * (1 + ze * ua)
                    dz = 0.25 * ua * (1 + xi * sa) * (1 + et * ta)
                    B[0, 3 * a], B[1, 3 * a + 1], B[2, 3 * a + 2] = dx, dy, dz
                    B[3, 3 * a], B[3, 3 * a + 1] = dy, dx
                    B[4, 3 * a + 1], B[4, 3 * a + 2] = dz, dy
                    B[5, 3 * a], B[5, 3 * a + 2] = dz, dx
                K += B.T @ D @ B * 0.125
    return K


def elasticity_q1(ex, ey, ez, contrast=1.0, nu=0.3, seed=42, permute=True):
    """Restatement of amg_gen_elasticity_q1 (gen.cpp): Q1 elasticity, x = 0 face
    clamped, per-element E = 10^(contrast (2u - 1)), seeded node permutation;
    3 dofs per node interleaved.  Returns scipy CSR."""
    nx, ny, nz = ex + 1, ey + 1, ez + 1
    nfree = ex * ny * nz
    ids = -np.ones(nx * ny * nz, np.int64)
    k = 0
    for z in range(nz):
        for y in range(ny):
            for x in range(1, nx):
                ids[x + nx * (y + ny * z)] = k
                k += 1
    if permute:
        W = nfree if permute is True or permute == 1 else int(permute)
        perm = list(range(nfree))
        M = (1 << 64) - 1
        a = _splitmix64(seed ^ 0xA5A5A5A5)
        for w0 in range(0, nfree, W):
            m = min(W, nfree - w0)
            for i in range(m - 1, 0, -1):
                r = a ^ _splitmix64((seed + 7 * (w0 + i)) & M)
                j = r % (i + 1)
                perm[w0 + i], perm[w0 + j] = perm[w0 + j], perm[w0 + i]
        perm = np.array(perm)
        ids = np.where(ids >= 0, perm[np.maximum(ids, 0)], -1)
    K = q1_reference_stiffness(nu)
    rows, cols, vals = [], [], []
    for z in range(ez):
        for y in range(ey):
            for x in range(ex):
                e = x + ex * (y + ey * z)
                E = 10.0 ** (contrast * (2.0 * _unit(seed, e) - 1.0))
                node = [ids[(x + (a & 1)) + nx * ((y + ((a >> 1) & 1)) + ny * (z + ((a >> 2) & 1)))]
                        for a in range(8)]
                for a in range(8):
                    if node[a] < 0:
                        continue
                    for b in range(8):
                        if node[b] < 0:
                            continue
                        for c in range(3):
                            for d in range(3):
                                rows.append(3 * node[a] + c)
                                cols.append(3 * node[b] + d)
                                vals.append(E * K[3 * a + c, 3 * b + d])
    n = 3 * nfree
    A = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()  # duplicates summed
    A.sort_indices()
    return A


# ------------------------------------------------------------------ strength

def strength_graph(A, nn, w, depth=1, block_size=1):
    """AdjacencyList::new_ls_strength_graph (partitioners/mod.rs:337-393) on the
    dof graph; block_size > 1: aggregate + filter_diag (:294-301, :464-497).
    Same operation order as sa.hip (theta 0.5, alpha 4, eps 1e-30 / 1e-12)."""
    A = A.tocsr()
    n = A.shape[0]
    nn = np.asarray(nn, np.float64).reshape(n, -1)
    k = nn.shape[1]
    w = [float(v) for v in w]
    NN = nn.tolist()

    def vnorm(i):
        s = 0.0
        for c in range(k):
            s += (NN[i][c] * w[c]) * NN[i][c]
        return max(s, 1e-30)

    vn = [vnorm(i) for i in range(n)]
    rp, ci = A.indptr, A.indices
    dof = []
    for i in range(n):
        if depth == 1:
            nb = [int(j) for j in ci[rp[i]:rp[i + 1]] if j != i]
        else:
            seen = {i}
            frontier, nb = [i], []
            for _ in range(depth):
                nxt = []
                for u in frontier:
                    for v in ci[rp[u]:rp[u + 1]]:
                        v = int(v)
                        if v not in seen:
                            seen.add(v)
                            nxt.append(v)
                            nb.append(v)
                frontier = nxt
        cand = []
        for j in nb:
            a, b = min(i, j), max(i, j)
            x = 0.0
            for c in range(k):
                x += (NN[a][c] * w[c]) * NN[b][c]
            rho2 = (x * x) / (vn[a] * vn[b])
            cand.append((2.0 * math.sqrt(max(1.0 - rho2, 0.0)), j))
        cand.sort()
        out = []
        if cand:
            keep = max(int(math.floor(len(cand) * 0.5)), 1)
            cand = cand[:keep]
            dmin, dmax = cand[0][0], cand[-1][0]
            for d, j in cand:
                wt = 1.0 if abs(dmax - dmin) < 1e-12 else math.pow((dmax - d) / (dmax - dmin + 1e-12), 4.0)
                out.append((j, wt))
            out.sort(key=lambda t: t[0])
        dof.append(out)
    if block_size == 1:
        return _lists_to_csr(dof, n)
    nnodes = n // block_size
    node, lmax = [], []
    for I in range(nnodes):
        cat = []
        for r in range(block_size):
            cat += [(j // block_size, v) for j, v in dof[I * block_size + r]]
        cat.sort(key=lambda t: t[0])  # stable
        out = []
        for j, v in cat:
            if out and out[-1][0] == j:
                out[-1] = (j, out[-1][1] + v)
            else:
                out.append((j, v))
        node.append(out)
        lmax.append(max([v for _, v in out], default=0.0))
    gmax = max(lmax)
    node = [[(j, v / gmax) for j, v in out if j != I] for I, out in enumerate(node)]
    return _lists_to_csr(node, nnodes)


def _lists_to_csr(lists, n):
    rp = np.zeros(n + 1, np.int64)
    for i, l in enumerate(lists):
        rp[i + 1] = rp[i] + len(l)
    ci = np.array([j for l in lists for j, _ in l], np.int64)
    va = np.array([v for l in lists for _, v in l], np.float64)
    return sp.csr_matrix((va, ci, rp), shape=(n, n))


def aggregate_mis(G):
    """Aggregates seeded by maximal_independent_set (partitioners/mod.rs:395-423),
    singleton roots joined to the strongest neighbour's aggregate (size >= 2),
    aggregates numbered by their smallest node (sa.hip)."""
    G = G.tocsr()
    n = G.shape[0]
    rp, ci, va = G.indptr, G.indices, G.data
    deg = []
    for i in range(n):
        s = 0.0
        for e in range(rp[i], rp[i + 1]):
            s += va[e]
        deg.append(s)
    order = sorted(range(n), key=lambda i: (-deg[i], i))
    agg = [-1] * n
    size, roots = [], []
    for i in order:
        if agg[i] >= 0:
            continue
        a = len(size)
        agg[i] = a
        size.append(1)
        roots.append(i)
        for e in range(rp[i], rp[i + 1]):
            j = ci[e]
            if agg[j] < 0:
                agg[j] = a
                size[a] += 1
    size0 = list(size)
    singles = sorted(roots[a] for a in range(len(roots)) if size0[a] == 1)
    for i in singles:
        best, bw = -1, -1.0
        for e in range(rp[i], rp[i + 1]):
            j = ci[e]
            if size0[agg[j]] < 2:
                continue
            if va[e] > bw or (va[e] == bw and j < best):
                bw, best = va[e], j
        if best >= 0:
            agg[i] = agg[best]
    ren, na = {}, 0
    out = np.zeros(n, np.int64)
    for i in range(n):
        if agg[i] not in ren:
            ren[agg[i]] = na
            na += 1
        out[i] = ren[agg[i]]
    return out, na


# ------------------------------------------------------------------ tentative P

def tentative_projectors(agg_of, naggs, nn, block_size, cd):
    """Per aggregate, the projector U_cd U_cd^T onto the first cd left singular
    vectors of the local near-null block (interpolation/mod.rs:754-805), via
    LAPACK SVD; basis-independent, so it checks P_J regardless of the sign /
    rotation the SVD of a degenerate block picks."""
    nn = np.asarray(nn).reshape(len(agg_of) * block_size, -1)
    out = []
    for a in range(naggs):
        nodes = np.flatnonzero(agg_of == a)
        rows = (nodes[:, None] * block_size + np.arange(block_size)).ravel()
        U, s, Vt = np.linalg.svd(nn[rows], full_matrices=False)
        Uc = U[:, :cd]
        out.append((rows, Uc @ Uc.T, s))
    return out


# ------------------------------------------------------------------ smoothing

def block_jacobi(A, P, block_size, omega=0.66):
    """block_jacobi (interpolation/mod.rs:963-1028): D^-1 per diagonal block by
    self_adjoint_eigen (lower triangle), P_s = (-omega D^-1)(A P) + P."""
    A = A.tocsr()
    n = A.shape[0]
    blocks = []
    for b in range(n // block_size):
        s = slice(b * block_size, (b + 1) * block_size)
        B = A[s, s].toarray()
        lam, U = np.linalg.eigh(np.tril(B) + np.tril(B, -1).T)
        assert np.all(lam > 1e-6)
        blocks.append(-omega * (U @ np.diag(1 / lam) @ U.T))
    Dinv = sp.block_diag(blocks, format="csr")
    return (Dinv @ (A @ P) + P).tocsr()


def smooth_interpolation(A, P, omega=0.66):
    """smooth_interpolation (interpolation/mod.rs:927-946)."""
    A = A.tocsr()
    d = A.diagonal()
    return (sp.diags(-omega / d) @ (A @ P) + P).tocsr()


def nn_postprocess(A, x, iters=3):
    """hierarchy.rs:219-228: StationaryIteration(L1, iters) per column with the
    r = x - A x quirk (smoothers.rs:146-158), then thin QR (R diag > 0)."""
    A = A.tocsr()
    d = 1.0 / np.asarray(abs(A).sum(axis=1)).ravel()
    x = np.array(x, np.float64, copy=True).reshape(A.shape[0], -1)
    for c in range(x.shape[1]):
        v = d * x[:, c]
        for _ in range(1, iters):
            v = v + d * (v - A @ v)
        x[:, c] = v
    Q, R = np.linalg.qr(x)
    return Q * np.sign(np.diag(R))


# ------------------------------------------------------- general 7-pt operator

_M64 = (1 << 64) - 1


def _edge_w(seed, a, b):
    lo, hi = min(a, b), max(a, b)
    h = _splitmix64((seed ^ _splitmix64((lo * 0x9E3779B97F4A7C15 + hi) & _M64)) & _M64)
    return 0.5 + float(h >> 11) * 2.0 ** -53


def _feistel(v, h, seed, key, inv):
    mask = (1 << h) - 1
    L, R = v >> h, v & mask
    for k in range(4):
        rk = 3 - k if inv else k
        x = seed ^ ((key * 0xD1B54A32D192ED03) & _M64) ^ (rk << 56) ^ (L if inv else R)
        f = _splitmix64(x & _M64) & mask
        if not inv:
            L, R = R, L ^ f
        else:
            L, R = R ^ f, L
    return (L << h) | R


def _perm(i, n, window, h, seed, inv):
    if window < 0:
        return i
    W = n if window == 0 else window
    w = i // W
    base = w * W
    m = min(W, n - base)
    hh = h
    while (1 << (2 * hh)) >= 4 * m and hh > 1:
        hh -= 1
    u = i - base
    while True:
        u = _feistel(u, hh, seed, w, inv)
        if u < m:
            return base + u


def random_7pt(nx, ny, nz, seed=42, window=4096):
    """Restatement of amg_gen_random_7pt (csr.hip): edge weights 0.5 + U[0,1),
    Dirichlet diagonal, symmetric permutation by 4-round Feistel bijections
    with cycle walking.  Returns scipy CSR (columns ascending)."""
    n = nx * ny * nz
    W = n if window == 0 else window
    h = 1
    while (1 << (2 * h)) < W:
        h += 1
    rows, cols, vals = [], [], []
    for r in range(n):
        i = _perm(r, n, window, h, seed, True)
        x, y, z = i % nx, (i // nx) % ny, i // (nx * ny)
        nb = [i - 1 if x > 0 else -1, i + 1 if x + 1 < nx else -1, i - nx if y > 0 else -1,
              i + nx if y + 1 < ny else -1, i - nx * ny if z > 0 else -1, i + nx * ny if z + 1 < nz else -1]
        diag = 0.0
        for j in nb:
            if j < 0:
                diag = diag + 1.0
                continue
            w = _edge_w(seed, i, j)
            diag = diag + w
            rows.append(r)
            cols.append(_perm(j, n, window, h, seed, False))
            vals.append(-w)
        rows.append(r)
        cols.append(r)
        vals.append(diag)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    A.sort_indices()
    return A
