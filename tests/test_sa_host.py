"""Host-side pieces of the general SA setup (config C5) against the Python
restatement in oracle/sa_oracle.py -- no GPU needed.

  * amg_gen_elasticity_q1 (gen.cpp), the in-tree Flan_1565 stand-in: pattern
    identical, values to 1e-13 of the row scale (the element matrix is summed
    in a different order by numpy's B^T D B), symmetric, SPD.
  * amg_aggregate_mis (sa.hip) on strength graphs built by the restatement:
    aggregates identical (same summation order, same tie rules).
Parity unpinned: the reference has no fixtures for these.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import sa_oracle as SO


def fa():
    import faer_amg_amd
    return faer_amg_amd


@pytest.mark.parametrize("elements,permute", [((3, 2, 4), False), ((4, 3, 3), True), ((5, 3, 3), 13)])
def test_elasticity_generator(elements, permute):
    H = fa().elasticity_q1(elements, contrast=1.0, nu=0.3, seed=7, permute=permute)
    G = H.to_scipy()
    R = SO.elasticity_q1(*elements, contrast=1.0, nu=0.3, seed=7, permute=permute)
    assert G.shape == R.shape
    assert np.array_equal(G.indptr, R.indptr) and np.array_equal(G.indices, R.indices)
    scale = abs(R).max()
    assert np.max(np.abs(G.data - R.data)) <= 1e-13 * scale
    assert abs(G - G.T).max() <= 1e-14 * scale
    ex, ey, ez = elements
    assert G.shape[0] == 3 * ex * (ey + 1) * (ez + 1)   # x = 0 face clamped
    assert np.linalg.eigvalsh(G.toarray()).min() > 0
    # 27-node couplings in the interior: 81 entries per row at most
    assert np.diff(G.indptr).max() == 81 or min(elements) < 2


def test_elasticity_generator_is_unstructured():
    """The permuted numbering spreads columns: no fixed set of diagonals."""
    G = fa().elasticity_q1((6, 6, 6), seed=3, permute=True).to_scipy().tocoo()
    offs = np.unique(G.col - G.row)
    assert len(offs) > 1000


def _graph_of(elements, seed, bs_nodes=True):
    A = SO.elasticity_q1(*elements, seed=seed)
    n = A.shape[0]
    nn = np.zeros((n, 3))
    for c in range(3):
        nn[c::3, c] = 1.0
    nn /= np.sqrt(n // 3)
    w = [1.0 / float(nn[:, c] @ (A @ nn[:, c])) for c in range(3)]
    return SO.strength_graph(A, nn, w, depth=1, block_size=3 if bs_nodes else 1)


@pytest.mark.parametrize("elements,seed", [((4, 3, 3), 1), ((5, 4, 3), 2)])
def test_aggregate_mis_matches_restatement(elements, seed):
    G = _graph_of(elements, seed)
    agg, na = fa().aggregate_mis(G)
    ragg, rna = SO.aggregate_mis(G)
    assert na == rna and np.array_equal(agg, ragg)
    # every aggregate non-empty, numbered by its smallest node
    first = [np.flatnonzero(agg == a)[0] for a in range(na)]
    assert first == sorted(first)
    assert na < G.shape[0]


def test_aggregate_mis_random_graph():
    """Asymmetric random strengths with ties and isolated nodes."""
    rng = np.random.default_rng(5)
    n = 300
    M = sp.random(n, n, density=0.02, random_state=rng, format="csr")
    M.data = np.round(M.data * 4) / 4 + 0.25   # many equal weights
    M.setdiag(0)
    M.eliminate_zeros()
    M.sort_indices()
    agg, na = fa().aggregate_mis(M)
    ragg, rna = SO.aggregate_mis(M)
    assert na == rna and np.array_equal(agg, ragg)
