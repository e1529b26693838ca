// sa.hip -- smoothed-aggregation setup for general (unstructured, block) SPD
// matrices: the path config C5 (Flan_1565-class elasticity, block size 3, three
// candidates) needs, where sa_build_box (ops.hip) only covers structured grids
// with one constant candidate.
//
// Restated from the reference (paths relative to its root):
//  * strength graph        AdjacencyList::new_ls_strength_graph
//                          (partitioners/mod.rs:337-393), block reduction
//                          aggregate + filter_diag (:294-301, :464-497)
//  * aggregation           stand-in for the modularity partitioner (OUT of
//                          scope): aggregates seeded by the
//                          reference's own maximal_independent_set
//                          (partitioners/mod.rs:395-423) -- every root claims
//                          its still-free strong neighbours
//  * tentative P           smoothed_aggregation (interpolation/mod.rs:754-805):
//                          per-aggregate thin SVD of the local near-null block,
//                          P = first `candidate_dimension` left singular
//                          vectors, coarse near-null = S V^T rows
//  * P smoothing           smooth_interpolation (:927-946) for block size 1,
//                          block_jacobi (:963-1028) otherwise
//  * R = P^T, A_c = R (A P) (:824-828) on the device (spgemm.hip)
//  * coarse near-null      StationaryIteration(L1, 3) with the r = x - A x
//                          quirk, then thin QR (hierarchy.rs:219-228)
//  * level loop            Hierarchy::coarsen (hierarchy.rs:190-248); the
//                          coarse block size is the candidate dimension
//                          (:210-213); the fine near-null weights are used on
//                          every level (the reference never pushes new ones).
// Determinism rules the reference leaves to unstable sorts are fixed here:
// ties in strength are broken by column, ties in MIS degree by node index.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <numeric>

#include "handles.hpp"

namespace famg {

// ------------------------------------------------------------ host helpers

struct HostPattern {
    int64_t n = 0;
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
};

static HostPattern download_pattern(const GpuCsr &m) {
    HostPattern h;
    h.n = m.nrows;
    h.rp.resize(m.nrows + 1);
    h.col.resize(m.nnz);
    hipStream_t s = m.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(h.rp.data(), m.rp64.get(), (m.nrows + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (m.nnz)
        FAMG_CHECK_HIP(hipMemcpyAsync(h.col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return h;
}

// ------------------------------------------------------------ strength graph

// new_ls_strength_graph (partitioners/mod.rs:337-393) on the dof graph, then
// (block_size > 1) merged to nodes (:294-301).  near-null: n x k column-major
// with leading dimension ld; weights: k entries (the diagonal W).
StrengthGraph strength_graph(const CsrOp &A, const double *nn, int64_t ld, int64_t k, const double *w,
                             int64_t depth, int64_t bs) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "strength graph: matrix must be square");
    FAMG_REQUIRE(bs >= 1 && A.nrows % bs == 0, AMG_ERR_DIM, "strength graph: block size must divide n");
    FAMG_REQUIRE(k >= 1 && ld >= A.nrows && depth >= 1, AMG_ERR_INVALID, "strength graph: bad near-null/depth");
    const int64_t n = A.nrows;
    const HostPattern pat = download_pattern(A.m);
    // v_i W v_i^T, floored at eps = 1e-30 (:352,355)
    std::vector<double> vn(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        double s = 0.0;
        for (int64_t c = 0; c < k; c++) s += (nn[i + c * ld] * w[c]) * nn[i + c * ld];
        vn[i] = std::max(s, 1e-30);
    }
    // per dof: kept neighbours (column ascending) and their strengths
    std::vector<std::vector<std::pair<int32_t, double>>> dof(n);
#pragma omp parallel
    {
        std::vector<int64_t> stamp(depth > 1 ? n : 0, -1);
        std::vector<int32_t> frontier, next, nb;
        std::vector<std::pair<double, int32_t>> cand;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < n; i++) {
            nb.clear();
            if (depth == 1) {
                for (int64_t e = pat.rp[i]; e < pat.rp[i + 1]; e++)
                    if (pat.col[e] != i) nb.push_back(pat.col[e]);
            } else {  // extract_local_subgraph (partitioners/mod.rs:695-718): BFS to `depth`
                stamp[i] = i;
                frontier.assign(1, (int32_t)i);
                for (int64_t d = 0; d < depth && !frontier.empty(); d++) {
                    next.clear();
                    for (int32_t u : frontier)
                        for (int64_t e = pat.rp[u]; e < pat.rp[u + 1]; e++) {
                            const int32_t v = pat.col[e];
                            if (stamp[v] != i) {
                                stamp[v] = i;
                                next.push_back(v);
                                nb.push_back(v);
                            }
                        }
                    frontier.swap(next);
                }
            }
            cand.clear();
            for (int32_t j : nb) {
                // the pair is always evaluated as (min, max): one value per edge (:353-360)
                const int64_t a = std::min<int64_t>(i, j), b = std::max<int64_t>(i, j);
                double x = 0.0;
                for (int64_t c = 0; c < k; c++) x += (nn[a + c * ld] * w[c]) * nn[b + c * ld];
                const double rho2 = (x * x) / (vn[a] * vn[b]);
                cand.push_back({2.0 * std::sqrt(std::max(1.0 - rho2, 0.0)), j});
            }
            // keep the strongest half (theta = 0.5), at least one (:367-373)
            std::sort(cand.begin(), cand.end());
            auto &out = dof[i];
            if (!cand.empty()) {
                const size_t keep = std::max<size_t>((size_t)std::floor((double)cand.size() * 0.5), 1);
                cand.resize(keep);
                const double dmin = cand.front().first, dmax = cand.back().first;
                out.reserve(keep);
                for (auto &cd : cand) {
                    double wt;
                    if (std::fabs(dmax - dmin) < 1e-12) wt = 1.0;
                    else wt = std::pow((dmax - cd.first) / (dmax - dmin + 1e-12), 4.0);  // alpha = 4 (:365,384-385)
                    out.push_back({cd.second, wt});
                }
                std::sort(out.begin(), out.end(),
                          [](const std::pair<int32_t, double> &p, const std::pair<int32_t, double> &q) {
                              return p.first < q.first;
                          });
            }
        }
    }
    StrengthGraph G;
    if (bs == 1) {
        G.n = n;
        G.rp.assign(n + 1, 0);
        for (int64_t i = 0; i < n; i++) G.rp[i + 1] = G.rp[i] + (int64_t)dof[i].size();
        G.col.resize(G.rp[n]);
        G.w.resize(G.rp[n]);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++) {
            int64_t o = G.rp[i];
            for (auto &p : dof[i]) { G.col[o] = p.first; G.w[o] = p.second; o++; }
        }
        return G;
    }
    // block reduction: node I merges the lists of its bs dofs, neighbour ids
    // j / bs, weights of equal ids summed in dof order; all divided by the
    // largest merged weight (self loops included, :476-490); then self loops
    // dropped (filter_diag, :493-497)
    const int64_t nn_nodes = n / bs;
    std::vector<std::vector<std::pair<int32_t, double>>> node(nn_nodes);
    std::vector<double> lmax(nn_nodes, 0.0);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t I = 0; I < nn_nodes; I++) {
        std::vector<std::pair<int32_t, double>> cat;
        for (int64_t r = 0; r < bs; r++)
            for (auto &p : dof[I * bs + r]) cat.push_back({(int32_t)(p.first / bs), p.second});
        std::stable_sort(cat.begin(), cat.end(),
                         [](const std::pair<int32_t, double> &p, const std::pair<int32_t, double> &q) {
                             return p.first < q.first;
                         });
        auto &out = node[I];
        for (auto &p : cat) {
            if (!out.empty() && out.back().first == p.first) out.back().second += p.second;
            else out.push_back(p);
        }
        double m = 0.0;
        for (auto &p : out) m = std::max(m, p.second);
        lmax[I] = m;
    }
    const double gmax = *std::max_element(lmax.begin(), lmax.end());
    FAMG_REQUIRE(gmax > 0.0, AMG_ERR_INVALID, "strength graph has no edges");
    G.n = nn_nodes;
    G.rp.assign(nn_nodes + 1, 0);
    for (int64_t I = 0; I < nn_nodes; I++) {
        int64_t c = 0;
        for (auto &p : node[I]) c += p.first != I;
        G.rp[I + 1] = G.rp[I] + c;
    }
    G.col.resize(G.rp[nn_nodes]);
    G.w.resize(G.rp[nn_nodes]);
#pragma omp parallel for schedule(static)
    for (int64_t I = 0; I < nn_nodes; I++) {
        int64_t o = G.rp[I];
        for (auto &p : node[I])
            if (p.first != I) { G.col[o] = p.first; G.w[o] = p.second / gmax; o++; }
    }
    return G;
}

// ------------------------------------------------------------ aggregation

// Aggregates seeded by maximal_independent_set (partitioners/mod.rs:395-423):
// nodes in descending strength degree (ties: ascending index); a node still
// free becomes a root and claims every still-free neighbour.  A root that
// claimed nothing joins the aggregate (of size >= 2) of its strongest
// neighbour.  Aggregates are numbered by their smallest node.
int64_t aggregate_mis(const StrengthGraph &G, std::vector<int64_t> &agg_of) {
    const int64_t n = G.n;
    std::vector<double> deg(n, 0.0);
    for (int64_t i = 0; i < n; i++)
        for (int64_t e = G.rp[i]; e < G.rp[i + 1]; e++) deg[i] += G.w[e];
    std::vector<int64_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return deg[a] > deg[b]; });
    std::vector<int64_t> agg(n, -1), size;
    std::vector<int64_t> roots;
    for (int64_t i : order) {
        if (agg[i] >= 0) continue;
        const int64_t a = (int64_t)size.size();
        agg[i] = a;
        size.push_back(1);
        roots.push_back(i);
        for (int64_t e = G.rp[i]; e < G.rp[i + 1]; e++) {
            const int64_t j = G.col[e];
            if (agg[j] < 0) { agg[j] = a; size[a]++; }
        }
    }
    // singleton roots: join the strongest neighbour's aggregate (size >= 2 before any merge)
    const std::vector<int64_t> size0 = size;
    std::vector<int64_t> singles;
    for (int64_t a = 0; a < (int64_t)roots.size(); a++)
        if (size0[a] == 1) singles.push_back(roots[a]);
    std::sort(singles.begin(), singles.end());
    for (int64_t i : singles) {
        int64_t best = -1;
        double bw = -1.0;
        for (int64_t e = G.rp[i]; e < G.rp[i + 1]; e++) {
            const int64_t j = G.col[e];
            if (size0[agg[j]] < 2) continue;
            if (G.w[e] > bw || (G.w[e] == bw && j < best)) { bw = G.w[e]; best = j; }
        }
        if (best >= 0) {
            size[agg[i]]--;
            agg[i] = agg[best];
        }
    }
    // renumber live aggregates by their smallest node
    std::vector<int64_t> ren(size.size(), -1);
    int64_t na = 0;
    for (int64_t i = 0; i < n; i++)
        if (ren[agg[i]] < 0) ren[agg[i]] = na++;
    agg_of.resize(n);
    for (int64_t i = 0; i < n; i++) agg_of[i] = ren[agg[i]];
    return na;
}

// ------------------------------------------------------------ tentative P

// Thin SVD of a rows x k matrix M (column-major, ld rows) by one-sided Jacobi:
// U (rows x k, columns ordered by descending singular value), s (k), V (k x k,
// column-major).  Zero singular directions get an orthonormal completion.
static void thin_svd(int64_t rows, int64_t k, const double *M, std::vector<double> &U, std::vector<double> &s,
                     std::vector<double> &V) {
    std::vector<double> u(M, M + rows * k), v(k * k, 0.0);
    for (int64_t c = 0; c < k; c++) v[c * k + c] = 1.0;
    for (int sweep = 0; sweep < 60 && k > 1; sweep++) {
        bool rotated = false;
        for (int64_t p = 0; p < k - 1; p++)
            for (int64_t q = p + 1; q < k; q++) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int64_t r = 0; r < rows; r++) {
                    al += u[p * rows + r] * u[p * rows + r];
                    be += u[q * rows + r] * u[q * rows + r];
                    ga += u[p * rows + r] * u[q * rows + r];
                }
                if (std::fabs(ga) <= 1e-15 * std::sqrt(al * be) || ga == 0.0) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
                for (int64_t r = 0; r < rows; r++) {
                    const double a = u[p * rows + r], b = u[q * rows + r];
                    u[p * rows + r] = c * a - sn * b;
                    u[q * rows + r] = sn * a + c * b;
                }
                for (int64_t r = 0; r < k; r++) {
                    const double a = v[p * k + r], b = v[q * k + r];
                    v[p * k + r] = c * a - sn * b;
                    v[q * k + r] = sn * a + c * b;
                }
            }
        if (!rotated) break;
    }
    std::vector<double> sig(k);
    for (int64_t c = 0; c < k; c++) {
        double ss = 0.0;
        for (int64_t r = 0; r < rows; r++) ss += u[c * rows + r] * u[c * rows + r];
        sig[c] = std::sqrt(ss);
    }
    std::vector<int64_t> ord(k);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return sig[a] > sig[b]; });
    U.assign(rows * k, 0.0);
    s.assign(k, 0.0);
    V.assign(k * k, 0.0);
    const double tiny = (k ? sig[ord[0]] : 0.0) * 1e-14;
    for (int64_t c = 0; c < k; c++) {
        const int64_t o = ord[c];
        s[c] = sig[o];
        for (int64_t r = 0; r < k; r++) V[c * k + r] = v[o * k + r];
        if (sig[o] > tiny && sig[o] > 0.0) {
            for (int64_t r = 0; r < rows; r++) U[c * rows + r] = u[o * rows + r] / sig[o];
        } else if (c < rows) {
            // orthonormal completion: the first unit vector independent of the columns so far
            for (int64_t e = 0; e < rows; e++) {
                std::vector<double> x(rows, 0.0);
                x[e] = 1.0;
                for (int pass = 0; pass < 2; pass++)
                    for (int64_t b = 0; b < c; b++) {
                        double d = 0.0;
                        for (int64_t r = 0; r < rows; r++) d += U[b * rows + r] * x[r];
                        for (int64_t r = 0; r < rows; r++) x[r] -= d * U[b * rows + r];
                    }
                double nx = 0.0;
                for (int64_t r = 0; r < rows; r++) nx += x[r] * x[r];
                nx = std::sqrt(nx);
                if (nx > 1e-8) {
                    for (int64_t r = 0; r < rows; r++) U[c * rows + r] = x[r] / nx;
                    break;
                }
            }
        }
    }
}

// smoothed_aggregation's tentative interpolation (interpolation/mod.rs:754-805)
// for `nnodes` nodes of `bs` dofs; coarse_nn: (naggs*cd) x k, column-major, ld
// naggs*cd.
CsrPtr sa_tentative_block(Ctx *ctx, int64_t nnodes, int64_t bs, const int64_t *agg_of, int64_t naggs,
                          const double *nn, int64_t ld, int64_t k, int64_t cd, double *coarse_nn) {
    FAMG_REQUIRE(bs >= 1 && k >= 1 && cd >= 1 && cd <= k && ld >= nnodes * bs, AMG_ERR_INVALID,
                 "tentative P: need block size >= 1, 1 <= candidate_dimension <= candidates");
    const int64_t n = nnodes * bs, ncd = naggs * cd;
    // nodes of each aggregate, ascending (BTreeSet order)
    std::vector<int64_t> aptr(naggs + 1, 0), anodes(nnodes);
    for (int64_t i = 0; i < nnodes; i++) {
        FAMG_REQUIRE(agg_of[i] >= 0 && agg_of[i] < naggs, AMG_ERR_INVALID, "node not aggregated");
        aptr[agg_of[i] + 1]++;
    }
    for (int64_t a = 0; a < naggs; a++) {
        FAMG_REQUIRE(aptr[a + 1] > 0, AMG_ERR_INVALID, "empty aggregate");
        aptr[a + 1] += aptr[a];
    }
    {
        std::vector<int64_t> pos(aptr.begin(), aptr.end() - 1);
        for (int64_t i = 0; i < nnodes; i++) anodes[pos[agg_of[i]]++] = i;
    }
    std::vector<int64_t> rp(n + 1), col(n * cd);
    std::vector<double> val(n * cd);
    for (int64_t i = 0; i <= n; i++) rp[i] = i * cd;
    std::atomic<bool> ok{true};  // written by the OpenMP threads
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t a = 0; a < naggs; a++) {
        const int64_t na = aptr[a + 1] - aptr[a], rows = na * bs;
        if (rows < cd) { ok.store(false, std::memory_order_relaxed); continue; }  // the reference asserts (:757-762)
        std::vector<double> M(rows * k), U, s, V;
        for (int64_t li = 0; li < na; li++) {
            const int64_t node = anodes[aptr[a] + li];
            for (int64_t o = 0; o < bs; o++)
                for (int64_t c = 0; c < k; c++) M[c * rows + li * bs + o] = nn[node * bs + o + c * ld];
        }
        thin_svd(rows, k, M.data(), U, s, V);
        // coarse near-null rows a*cd .. a*cd+cd-1 = (S V^T)[0..cd, :]
        for (int64_t q = 0; q < cd; q++)
            for (int64_t c = 0; c < k; c++) coarse_nn[a * cd + q + c * ncd] = s[q] * V[q * k + c];
        for (int64_t li = 0; li < na; li++) {
            const int64_t node = anodes[aptr[a] + li];
            for (int64_t o = 0; o < bs; o++) {
                const int64_t row = node * bs + o;
                for (int64_t q = 0; q < cd; q++) {
                    col[row * cd + q] = a * cd + q;
                    val[row * cd + q] = U[q * rows + li * bs + o];
                }
            }
        }
    }
    FAMG_REQUIRE(ok, AMG_ERR_INVALID, "an aggregate has fewer dofs than the candidate dimension");
    auto P = make_csr(ctx);
    csr_from_host(P->m, ctx, n, ncd, rp.data(), col.data(), val.data());
    P->nrows = n;
    P->ncols = ncd;
    return P;
}

// ------------------------------------------------------------ P smoothing

// diagonal blocks: out[i*bs + c] = a(i, (i/bs)*bs + c)
__global__ void k_block_diag(const int64_t *rp, const int32_t *col, const double *val, int64_t n, int64_t bs,
                             double *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t b0 = (i / bs) * bs;
    for (int64_t c = 0; c < bs; c++) out[i * bs + c] = 0.0;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        const int64_t j = col[e];
        if (j >= b0 && j < b0 + bs) out[i * bs + (j - b0)] = val[e];
    }
}

// S += P where P's pattern lies within S's (columns sorted in both)
__global__ void k_add_into(const int64_t *srp, const int32_t *scol, double *sval, const int64_t *prp,
                           const int32_t *pcol, const double *pval, int64_t m, int *bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int64_t s0 = srp[i], s1 = srp[i + 1];
    for (int64_t e = prp[i]; e < prp[i + 1]; e++) {
        int64_t lo = s0, hi = s1;
        const int32_t j = pcol[e];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (scol[mid] < j) lo = mid + 1;
            else hi = mid;
        }
        if (lo >= s1 || scol[lo] != j) { *bad = 1; return; }
        sval[lo] = sval[lo] + pval[e];
    }
}

void csr_add_into(GpuCsr &S, const GpuCsr &P) {
    FAMG_REQUIRE(S.nrows == P.nrows && S.ncols == P.ncols, AMG_ERR_DIM, "csr_add_into: shapes differ");
    hipStream_t s = S.ctx->stream;
    DevBuf<int> bad(1);
    FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
    if (S.nrows)
        hipLaunchKernelGGL(k_add_into, dim3((unsigned)ceil_div(S.nrows, 256)), dim3(256), 0, s, S.rp64.get(),
                           S.col.get(), S.val.get(), P.rp64.get(), P.col.get(), P.val.get(), S.nrows, bad.get());
    FAMG_CHECK_HIP(hipGetLastError());
    int h = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&h, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    FAMG_REQUIRE(h == 0, AMG_ERR_INVALID, "csr_add_into: pattern of the addend not within the sum");
}

// Symmetric eigen-decomposition of a bs x bs matrix (cyclic Jacobi; lower
// triangle read, as self_adjoint_eigen(Side::Lower)); returns U S^-1 U^T.
static bool block_inverse_eig(int64_t bs, const double *lower_rowmajor, double *inv) {
    std::vector<double> a(bs * bs), u(bs * bs, 0.0);
    for (int64_t i = 0; i < bs; i++)
        for (int64_t j = 0; j <= i; j++) a[i * bs + j] = a[j * bs + i] = lower_rowmajor[i * bs + j];
    for (int64_t i = 0; i < bs; i++) u[i * bs + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0;
        for (int64_t p = 0; p < bs; p++)
            for (int64_t q = p + 1; q < bs; q++) off += a[p * bs + q] * a[p * bs + q];
        if (off == 0.0) break;
        for (int64_t p = 0; p < bs - 1; p++)
            for (int64_t q = p + 1; q < bs; q++) {
                const double apq = a[p * bs + q];
                if (apq == 0.0) continue;
                const double theta = (a[q * bs + q] - a[p * bs + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int64_t r = 0; r < bs; r++) {  // A <- J^T A J
                    const double arp = a[r * bs + p], arq = a[r * bs + q];
                    a[r * bs + p] = c * arp - s * arq;
                    a[r * bs + q] = s * arp + c * arq;
                }
                for (int64_t r = 0; r < bs; r++) {
                    const double apr = a[p * bs + r], aqr = a[q * bs + r];
                    a[p * bs + r] = c * apr - s * aqr;
                    a[q * bs + r] = s * apr + c * aqr;
                }
                for (int64_t r = 0; r < bs; r++) {
                    const double urp = u[r * bs + p], urq = u[r * bs + q];
                    u[r * bs + p] = c * urp - s * urq;
                    u[r * bs + q] = s * urp + c * urq;
                }
            }
    }
    for (int64_t q = 0; q < bs; q++)
        if (!(a[q * bs + q] > 1e-6)) return false;  // the reference asserts (:999-1004)
    for (int64_t i = 0; i < bs; i++)
        for (int64_t j = 0; j < bs; j++) {
            double t = 0.0;
            for (int64_t q = 0; q < bs; q++) t += u[i * bs + q] * (1.0 / a[q * bs + q]) * u[j * bs + q];
            inv[i * bs + j] = t;
        }
    return true;
}

// block_jacobi (interpolation/mod.rs:963-1028): P_s = (-omega D^-1) (A P) + P,
// D = the bs x bs diagonal blocks of A.
CsrPtr block_jacobi_smooth(CsrOp &A, const CsrOp &P, int64_t bs, double omega) {
    FAMG_REQUIRE(A.nrows == A.ncols && A.ncols == P.nrows, AMG_ERR_DIM, "block_jacobi dims");
    FAMG_REQUIRE(bs >= 1 && A.nrows % bs == 0, AMG_ERR_DIM, "block_jacobi: block size must divide n");
    Ctx *ctx = A.ctx;
    hipStream_t s = ctx->stream;
    const int64_t n = A.nrows;
    DevBuf<double> dblk(std::max<int64_t>(1, n * bs));
    if (n)
        hipLaunchKernelGGL(k_block_diag, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, A.m.rp64.get(),
                           A.m.col.get(), A.m.val.get(), n, bs, dblk.get());
    FAMG_CHECK_HIP(hipGetLastError());
    std::vector<double> hb(n * bs);
    if (n) FAMG_CHECK_HIP(hipMemcpyAsync(hb.data(), dblk.get(), n * bs * sizeof(double), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    const int64_t nb = n / bs;
    std::vector<int64_t> rp(n + 1), col(n * bs);
    std::vector<double> val(n * bs);
    std::atomic<bool> ok{true};  // written by the OpenMP threads
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; b++) {
        std::vector<double> inv(bs * bs);
        if (!block_inverse_eig(bs, hb.data() + b * bs * bs, inv.data())) {
            ok.store(false, std::memory_order_relaxed);
            continue;
        }
        for (int64_t i = 0; i < bs; i++)
            for (int64_t j = 0; j < bs; j++) {
                col[(b * bs + i) * bs + j] = b * bs + j;
                val[(b * bs + i) * bs + j] = -omega * inv[i * bs + j];
            }
    }
    FAMG_REQUIRE(ok, AMG_ERR_NOT_SPD, "block_jacobi: a diagonal block is nearly singular (eigenvalue <= 1e-6)");
    for (int64_t i = 0; i <= n; i++) rp[i] = i * bs;
    auto Dinv = make_csr(ctx);
    csr_from_host(Dinv->m, ctx, n, n, rp.data(), col.data(), val.data());
    GpuCsr AP;
    spgemm(A.m, P.m, AP, false);
    GpuCsr S;
    spgemm(Dinv->m, AP, S, false);
    csr_add_into(S, P.m);
    csr_finalize(S);
    auto out = make_csr(ctx);
    out->m = std::move(S);
    out->nrows = n;
    out->ncols = P.ncols;
    return out;
}

// ------------------------------------------------------------ coarse near-null

__global__ void k_scale_by(double *x, const double *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = d[i] * x[i];
}

// hierarchy.rs:219-228 for k candidates: StationaryIteration(L1, iters) on every
// column (smoothers.rs:146-158, r = x - A x quirk), then thin QR (modified
// Gram-Schmidt with re-orthogonalisation; R's diagonal positive).  k = 1 is
// nn_stationary_l1 (the tree-reduced device norm the box builder uses).
void nn_postprocess(CsrOp &A, int64_t iters, double *x, int64_t ld, int64_t k) {
    const int64_t n = A.nrows;
    if (k == 1) {
        nn_stationary_l1(A, iters, x);
        return;
    }
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    auto d = make_l1(A);
    DevBuf<double> xd(std::max<int64_t>(1, n)), r(std::max<int64_t>(1, n));
    for (int64_t c = 0; c < k; c++) {
        if (!n) break;
        FAMG_CHECK_HIP(hipMemcpyAsync(xd.get(), x + c * ld, n * sizeof(double), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_scale_by, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, xd.get(), d->d.get(), n);
        for (int64_t it = 1; it < iters; it++) {
            spmv(A.m, xd.get(), r.get(), SPMV_SET, SpmvEpi{}, s);
            vec_nn_step(xd.get(), d->d.get(), r.get(), n, s);
        }
        FAMG_CHECK_HIP(hipMemcpyAsync(x + c * ld, xd.get(), n * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    for (int64_t c = 0; c < k; c++) {
        double *q = x + c * ld;
        for (int pass = 0; pass < 2; pass++)
            for (int64_t b = 0; b < c; b++) {
                const double *qb = x + b * ld;
                double dt = 0.0;
                for (int64_t i = 0; i < n; i++) dt += qb[i] * q[i];
                for (int64_t i = 0; i < n; i++) q[i] -= dt * qb[i];
            }
        double nr = 0.0;
        for (int64_t i = 0; i < n; i++) nr += q[i] * q[i];
        nr = std::sqrt(nr);
        FAMG_REQUIRE(nr > 0.0, AMG_ERR_INVALID, "coarse near-null space is rank deficient");
        for (int64_t i = 0; i < n; i++) q[i] /= nr;
    }
}

// ------------------------------------------------------------ hierarchy

// create_weights (examples/amg/main.rs:571-580): w_c = 1 / (v_c^T A v_c)
static std::vector<double> default_weights(CsrOp &A, const double *nn, int64_t ld, int64_t k) {
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    const int64_t n = A.nrows;
    DevBuf<double> v(std::max<int64_t>(1, n)), av(std::max<int64_t>(1, n));
    std::vector<double> w(k);
    for (int64_t c = 0; c < k; c++) {
        FAMG_CHECK_HIP(hipMemcpyAsync(v.get(), nn + c * ld, n * sizeof(double), hipMemcpyHostToDevice, s));
        spmv(A.m, v.get(), av.get(), SPMV_SET, SpmvEpi{}, s);
        const double vtav = vec_dot(v.get(), av.get(), n, ctx);
        FAMG_REQUIRE(vtav > 0.0, AMG_ERR_NOT_SPD, "near-null candidate with v^T A v <= 0");
        w[c] = 1.0 / vtav;
    }
    return w;
}

std::shared_ptr<MultigridOp> sa_build(const CsrPtr &A, const double *nn_in, int64_t ld, int64_t k,
                                      const double *weights_in, const SaConfig &cfg,
                                      std::vector<SaLevelInfo> *info) {
    FAMG_REQUIRE(A->nrows == A->ncols, AMG_ERR_DIM, "sa_build: matrix must be square");
    FAMG_REQUIRE(cfg.block_size >= 1 && A->nrows % cfg.block_size == 0, AMG_ERR_DIM,
                 "sa_build: block size must divide n");
    FAMG_REQUIRE(k >= 1 && cfg.candidate_dimension >= 1 && cfg.candidate_dimension <= k, AMG_ERR_INVALID,
                 "sa_build: need 1 <= candidate_dimension <= near-null columns");
    FAMG_REQUIRE(ld >= A->nrows, AMG_ERR_INVALID, "sa_build: near-null leading dimension < n");
    Ctx *ctx = A->ctx;
    const int64_t max_levels = cfg.max_levels <= 0 ? INT64_MAX : cfg.max_levels;
    const std::vector<double> w =
        weights_in ? std::vector<double>(weights_in, weights_in + k) : default_weights(*A, nn_in, ld, k);
    std::vector<CsrPtr> As{A}, Rs, Ps;
    std::vector<int64_t> bss{cfg.block_size};
    std::vector<std::vector<int64_t>> aggs;
    std::vector<int64_t> naggs;
    int64_t cur_ld = A->nrows;
    std::vector<double> nn(A->nrows * k);
    for (int64_t c = 0; c < k; c++) std::memcpy(nn.data() + c * cur_ld, nn_in + c * ld, A->nrows * sizeof(double));
    int64_t level = 1, coarse_dim = -1, bs = cfg.block_size;
    const int64_t cd = cfg.candidate_dimension;
    while ((coarse_dim < 0 || coarse_dim > cfg.coarsest_dim) && level < max_levels) {
        CsrPtr cur = As.back();
        const int64_t n = cur->nrows, nnodes = n / bs;
        StrengthGraph G = strength_graph(*cur, nn.data(), cur_ld, k, w.data(), cfg.strength_depth, bs);
        std::vector<int64_t> agg;
        const int64_t na = aggregate_mis(G, agg);
        if (na * cd >= n) break;  // no coarsening left (stall): stop here
        std::vector<double> cnn(na * cd * k);
        CsrPtr P = sa_tentative_block(ctx, nnodes, bs, agg.data(), na, nn.data(), cur_ld, k, cd, cnn.data());
        for (int64_t st = 0; st < cfg.smoothing_steps; st++)
            P = bs == 1 ? smooth_interpolation(*cur, *P, 0.66) : block_jacobi_smooth(*cur, *P, bs, 0.66);
        CsrPtr R = transpose_op(*P);
        CsrPtr Ac = galerkin_rap(*R, *cur, *P);
        nn_postprocess(*Ac, 3, cnn.data(), na * cd, k);
        if (info) info->push_back({n, bs, nnodes, na, G.rp.back()});
        aggs.push_back(std::move(agg));
        naggs.push_back(na);
        Rs.push_back(R);
        Ps.push_back(P);
        As.push_back(Ac);
        nn.swap(cnn);
        cur_ld = na * cd;
        bs = cd;
        bss.push_back(bs);
        coarse_dim = Ac->nrows;
        level++;
    }
    auto make_smoother = [&](const CsrPtr &M, size_t l) -> LinOpPtr {
        switch (cfg.smoother) {
        case 0: return make_jacobi(*M, cfg.omega);
        case 1: return make_l1(*M);
        case 2: {
            std::vector<int32_t> colors;
            const int64_t ncol = greedy_coloring(M->m, colors);
            if (ncol <= SGS_MAX_COLORS) return make_sgs(M, colors.data(), false);
            return make_l1(*M);
        }
        case 3:  // BlockSmoother over the level's aggregates (block_smoothers.rs)
            return make_block_smoother(*M, aggs[l].data(), naggs[l], bss[l]);
        default: fail(AMG_ERR_INVALID, "unknown smoother kind");
        }
    };
    auto mg = std::make_shared<MultigridOp>();
    mg->ctx = ctx;
    mg->nrows = mg->ncols = A->nrows;
    MgLevel L0;
    L0.A = A;
    L0.S = As.size() == 1 ? LinOpPtr(make_coarse_chol(*A)) : make_smoother(A, 0);
    mg->levels.push_back(std::move(L0));
    for (size_t l = 1; l < As.size(); l++) {
        LinOpPtr S = (l + 1 == As.size()) ? LinOpPtr(make_coarse_chol(*As[l])) : make_smoother(As[l], l);
        mg->add_level(As[l], S, Rs[l - 1], Ps[l - 1]);
    }
    return mg;
}

}  // namespace famg

// ------------------------------------------------------------------ C ABI

using namespace famg;

namespace {
CsrPtr need_csr_sa(const amg_linop *h) {
    FAMG_REQUIRE(h && h->op, AMG_ERR_INVALID, "null amg_linop handle");
    auto p = std::dynamic_pointer_cast<CsrOp>(h->op);
    FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not a CSR matrix");
    return p;
}
}  // namespace

extern "C" {

amg_status amg_sa_config_default(amg_sa_config *cfg) {
    return guard([&] {
        FAMG_REQUIRE(cfg, AMG_ERR_INVALID, "null config");
        std::memset(cfg, 0, sizeof(*cfg));
        cfg->block_size = 1;
        cfg->candidate_dimension = 1;
        cfg->strength_depth = 1;
        cfg->smoothing_steps = 1;     // AggregationConfig::default (interpolation/mod.rs:71-79)
        cfg->coarsest_dim = 1000;     // HierarchyConfig::default (hierarchy.rs:28-35)
        cfg->max_levels = 0;
        cfg->omega = 0.66;
        cfg->smoother = 1;
    });
}

amg_status amg_sa_build(amg_linop *A, const double *near_null, int64_t ld, int64_t k, const double *weights,
                        const amg_sa_config *cfg, amg_linop **mg_out) {
    return guard([&] {
        auto a = need_csr_sa(A);
        FAMG_REQUIRE(near_null && cfg && mg_out, AMG_ERR_INVALID, "null argument");
        a->ctx->set_device();
        SaConfig c;
        c.block_size = cfg->block_size;
        c.candidate_dimension = cfg->candidate_dimension;
        c.strength_depth = cfg->strength_depth;
        c.smoothing_steps = cfg->smoothing_steps;
        c.coarsest_dim = cfg->coarsest_dim;
        c.max_levels = cfg->max_levels;
        c.omega = cfg->omega;
        c.smoother = cfg->smoother;
        *mg_out = new amg_linop{sa_build(a, near_null, ld, k, weights, c, nullptr)};
    });
}

amg_status amg_strength_graph(const amg_linop *A, const double *near_null, int64_t ld, int64_t k,
                              const double *weights, int64_t depth, int64_t block_size, amg_host_csr **out) {
    return guard([&] {
        auto a = need_csr_sa(A);
        FAMG_REQUIRE(near_null && weights && out, AMG_ERR_INVALID, "null argument");
        a->ctx->set_device();
        StrengthGraph G = strength_graph(*a, near_null, ld, k, weights, depth, block_size);
        auto *h = new amg_host_csr;
        h->nrows = h->ncols = G.n;
        h->rp = std::move(G.rp);
        h->ci.assign(G.col.begin(), G.col.end());
        h->va = std::move(G.w);
        *out = h;
    });
}

amg_status amg_aggregate_mis(const amg_host_csr *graph, int64_t *agg_of, int64_t *naggs) {
    return guard([&] {
        FAMG_REQUIRE(graph && agg_of && naggs, AMG_ERR_INVALID, "null argument");
        FAMG_REQUIRE(graph->nrows == graph->ncols, AMG_ERR_DIM, "graph must be square");
        StrengthGraph G;
        G.n = graph->nrows;
        G.rp = graph->rp;
        G.col.assign(graph->ci.begin(), graph->ci.end());
        G.w = graph->va;
        std::vector<int64_t> agg;
        *naggs = aggregate_mis(G, agg);
        std::copy(agg.begin(), agg.end(), agg_of);
    });
}

amg_status amg_sa_tentative_block(amg_ctx *ctx, int64_t nnodes, int64_t block_size, const int64_t *agg_of,
                                  int64_t naggs, const double *near_null, int64_t ld, int64_t k, int64_t cd,
                                  amg_linop **P, double *coarse_nn) {
    return guard([&] {
        FAMG_REQUIRE(ctx && agg_of && near_null && P && coarse_nn && nnodes >= 0 && naggs > 0, AMG_ERR_INVALID,
                     "bad argument");
        Ctx *c = reinterpret_cast<Ctx *>(ctx);
        c->set_device();
        *P = new amg_linop{sa_tentative_block(c, nnodes, block_size, agg_of, naggs, near_null, ld, k, cd, coarse_nn)};
    });
}

amg_status amg_block_jacobi_smooth(const amg_linop *A, const amg_linop *P, int64_t block_size, double omega,
                                   amg_linop **out) {
    return guard([&] {
        auto a = need_csr_sa(A);
        auto p = need_csr_sa(P);
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        a->ctx->set_device();
        *out = new amg_linop{block_jacobi_smooth(*a, *p, block_size, omega)};
    });
}

amg_status amg_nn_postprocess(const amg_linop *A, int64_t iters, double *x, int64_t ld, int64_t k) {
    return guard([&] {
        auto a = need_csr_sa(A);
        FAMG_REQUIRE(x && k >= 1 && ld >= a->nrows && iters >= 1, AMG_ERR_INVALID, "bad argument");
        a->ctx->set_device();
        nn_postprocess(*a, iters, x, ld, k);
    });
}

}  // extern "C"
