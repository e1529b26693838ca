// block.hip -- BlockSmoother (preconditioners/block_smoothers.rs:80-291), the
// reference's default V-cycle smoother (MultigridConfig, multigrid.rs:42-49):
// block Jacobi over a partition of the nodes, each block the aggregate's
// diagonally compensated submatrix (diagonally_compensate, :293-324, and the
// vector form :326-400) solved exactly (BlockSolver(Cholesky), the default kind).
//
// Setup (host, OpenMP over blocks): compensated dense block -> Cholesky ->
// explicit inverse, stored column-major per block.  The reference solves each
// block with a sparse LL^T; the inverse is the same operator (rounding-level
// differences).  Apply (device): blocks are grouped into chunks of <= 256 rows
// (a larger block is a chunk of its own); one workgroup per chunk gathers the
// chunk's rhs entries into LDS, then thread i of a block computes
// out_i = sum_j inv[j][i] rhs_j (ascending j, fma) with lane-contiguous reads
// of inverse column j.  Every block is read completely before it is written,
// so apply_in_place needs no scratch.  Bytes per apply: 8 s_b^2 per block +
// 24 B per row (gather, scatter, index) -- HBM-bound; 64 B/row of inverse for
// 2^3 boxes (vs ~72 B/row for a 7-pt SpMV).
#include <algorithm>
#include <cmath>

#include "handles.hpp"

using namespace famg;

namespace famg {

constexpr int BLK_CHUNK = 256;
constexpr int64_t BLK_MAX = 8192;  // rows per block (LDS: 64 KB of rhs)

__global__ __launch_bounds__(BLK_CHUNK) void k_block_apply(const int32_t *rows, const int32_t *blk_of,
                                                           const int64_t *bptr, const int64_t *ioff,
                                                           const int32_t *chunk, const double *inv,
                                                           const double *r, double *out) {
    extern __shared__ double sr[];
    const int c = blockIdx.x;
    const int p0 = chunk[c], p1 = chunk[c + 1];
    for (int q = threadIdx.x; q < p1 - p0; q += BLK_CHUNK) sr[q] = r[rows[p0 + q]];
    __syncthreads();
    for (int q = threadIdx.x; q < p1 - p0; q += BLK_CHUNK) {
        const int p = p0 + q;
        const int b = blk_of[p];
        const int64_t b0 = bptr[b];
        const int s = (int)(bptr[b + 1] - b0);
        const int i = (int)(p - b0);
        const double *M = inv + ioff[b] + i;
        const double *x = sr + (b0 - p0);
        double acc = 0.0;
        for (int j = 0; j < s; j++) acc = fma(M[(int64_t)j * s], x[j], acc);
        out[rows[p]] = acc;
    }
}

void BlockSmootherOp::apply(double *out, const double *rhs) {
    if (nchunks == 0) return;
    const size_t lds = sizeof(double) * std::max<int64_t>(BLK_CHUNK, max_block);
    // inverses + rows/blk_of (8 B per row) + r gathered + out written
    log_launch("block", -1, -1, nrows, 8 * (int64_t)inv.size() + 24 * nrows);
    hipLaunchKernelGGL(k_block_apply, dim3((unsigned)nchunks), dim3(BLK_CHUNK), lds, ctx->stream, rows.get(),
                       blk_of.get(), bptr.get(), ioff.get(), chunk.get(), inv.get(), rhs, out);
    FAMG_CHECK_HIP(hipGetLastError());
}

namespace {

// dense SPD inverse (column-major in/out, s x s): Cholesky, then L^-T L^-1 e_j
bool spd_inverse(std::vector<double> &a, int64_t s, std::vector<double> &inv) {
    std::vector<double> L(a);  // column-major; use lower triangle
    auto at = [&](int64_t i, int64_t j) -> double & { return L[j * s + i]; };
    for (int64_t j = 0; j < s; j++) {
        double d = at(j, j);
        for (int64_t k = 0; k < j; k++) d -= at(j, k) * at(j, k);
        if (!(d > 0.0)) return false;
        const double ljj = std::sqrt(d);
        at(j, j) = ljj;
        for (int64_t i = j + 1; i < s; i++) {
            double t = at(i, j);
            for (int64_t k = 0; k < j; k++) t -= at(i, k) * at(j, k);
            at(i, j) = t / ljj;
        }
    }
    inv.assign(s * s, 0.0);
    std::vector<double> y(s);
    for (int64_t j = 0; j < s; j++) {
        std::fill(y.begin(), y.end(), 0.0);
        y[j] = 1.0;
        for (int64_t i = j; i < s; i++) {
            double t = y[i];
            for (int64_t k = j; k < i; k++) t -= at(i, k) * y[k];
            y[i] = t / at(i, i);
        }
        for (int64_t i = s - 1; i >= 0; i--) {
            double t = y[i];
            for (int64_t k = i + 1; k < s; k++) t -= at(k, i) * y[k];
            y[i] = t / at(i, i);
        }
        for (int64_t i = 0; i < s; i++) inv[j * s + i] = y[i];
    }
    return true;
}

// U S U^T of the SVD of M (v x v, row-major) = the PSD square root of M M^T,
// by cyclic Jacobi on M M^T.
void polar_u_s_ut(const std::vector<double> &M, int v, std::vector<double> &out) {
    std::vector<double> S(v * v, 0.0), Q(v * v, 0.0);
    for (int i = 0; i < v; i++)
        for (int j = 0; j < v; j++) {
            double t = 0.0;
            for (int k = 0; k < v; k++) t += M[i * v + k] * M[j * v + k];
            S[i * v + j] = t;
        }
    for (int i = 0; i < v; i++) Q[i * v + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0;
        for (int i = 0; i < v; i++)
            for (int j = i + 1; j < v; j++) off += S[i * v + j] * S[i * v + j];
        if (off < 1e-300) break;
        for (int p = 0; p < v; p++)
            for (int q = p + 1; q < v; q++) {
                const double apq = S[p * v + q];
                if (apq == 0.0) continue;
                const double theta = (S[q * v + q] - S[p * v + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < v; k++) {  // S = J^T S J
                    const double skp = S[k * v + p], skq = S[k * v + q];
                    S[k * v + p] = c * skp - sn * skq;
                    S[k * v + q] = sn * skp + c * skq;
                }
                for (int k = 0; k < v; k++) {
                    const double spk = S[p * v + k], sqk = S[q * v + k];
                    S[p * v + k] = c * spk - sn * sqk;
                    S[q * v + k] = sn * spk + c * sqk;
                }
                for (int k = 0; k < v; k++) {
                    const double qkp = Q[k * v + p], qkq = Q[k * v + q];
                    Q[k * v + p] = c * qkp - sn * qkq;
                    Q[k * v + q] = sn * qkp + c * qkq;
                }
            }
    }
    out.assign(v * v, 0.0);
    for (int i = 0; i < v; i++)
        for (int j = 0; j < v; j++) {
            double t = 0.0;
            for (int k = 0; k < v; k++) t += Q[i * v + k] * std::sqrt(std::max(0.0, S[k * v + k])) * Q[j * v + k];
            out[i * v + j] = t;
        }
}

}  // namespace

std::shared_ptr<BlockSmootherOp> make_block_smoother(CsrOp &A, const int64_t *part, int64_t nagg, int64_t vdim) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "block smoother: matrix must be square");
    FAMG_REQUIRE(vdim >= 1 && A.nrows % vdim == 0, AMG_ERR_DIM, "block size must divide the dimension");
    const int64_t n = A.nrows, nn = n / vdim;
    FAMG_REQUIRE(n < (int64_t(1) << 31), AMG_ERR_UNSUPPORTED, "block smoother needs n < 2^31");
    std::vector<int64_t> rp(n + 1), col(A.m.nnz);
    std::vector<double> val(A.m.nnz);
    csr_to_host(A.m, rp.data(), col.data(), val.data());
    // aggregates (nodes ascending, the BTreeSet order of the reference)
    std::vector<int64_t> cnt(nagg + 1, 0);
    for (int64_t i = 0; i < nn; i++) {
        FAMG_REQUIRE(part[i] >= 0 && part[i] < nagg, AMG_ERR_INVALID, "partition id out of range");
        cnt[part[i] + 1]++;
    }
    for (int64_t a = 0; a < nagg; a++) cnt[a + 1] += cnt[a];
    std::vector<int64_t> nodes(nn), pos(cnt.begin(), cnt.end() - 1);
    for (int64_t i = 0; i < nn; i++) nodes[pos[part[i]]++] = i;
    std::vector<int64_t> local(nn);  // node -> index within its aggregate
    for (int64_t a = 0; a < nagg; a++)
        for (int64_t k = cnt[a]; k < cnt[a + 1]; k++) local[nodes[k]] = k - cnt[a];
    std::vector<double> diag(n, 0.0);
    for (int64_t i = 0; i < n; i++)
        for (int64_t e = rp[i]; e < rp[i + 1]; e++)
            if (col[e] == i) diag[i] += val[e];
    auto op = std::make_shared<BlockSmootherOp>();
    op->ctx = A.ctx;
    op->nrows = op->ncols = n;
    op->vdim = vdim;
    op->nblocks = nagg;
    std::vector<int64_t> ioff(nagg + 1, 0), bptr(nagg + 1, 0);
    for (int64_t a = 0; a < nagg; a++) {
        const int64_t s = (cnt[a + 1] - cnt[a]) * vdim;
        FAMG_REQUIRE(s <= BLK_MAX, AMG_ERR_UNSUPPORTED, "block larger than 8192 rows");
        bptr[a + 1] = bptr[a] + s;
        ioff[a + 1] = ioff[a] + s * s;
        op->max_block = std::max(op->max_block, s);
    }
    std::vector<double> inv(ioff[nagg]);
    std::vector<int32_t> rows(n), blk_of(n);
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(| : bad)
    for (int64_t a = 0; a < nagg; a++) {
        const int64_t na = cnt[a + 1] - cnt[a], s = na * vdim;
        std::vector<double> B(s * s, 0.0);  // column-major
        auto in_agg = [&](int64_t node) { return part[node] == a; };
        if (vdim == 1) {
            // diagonally_compensate (block_smoothers.rs:293-324): row i adds, in
            // column order, a_ij for j in the aggregate and 0.5 sqrt(a_ii/a_jj)|a_ij|
            // to the diagonal otherwise
            for (int64_t k = 0; k < na; k++) {
                const int64_t i = nodes[cnt[a] + k];
                for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
                    const int64_t j = col[e];
                    if (in_agg(j)) B[local[j] * s + k] += val[e];
                    else B[k * s + k] += 0.5 * std::sqrt(diag[i] / diag[j]) * std::fabs(val[e]);
                }
            }
        } else {
            // diagonally_compensate_vector (:326-400): node-diagonal v x v blocks,
            // in-aggregate couplings, and 0.5 U S U^T of -A_IJ for every coupled
            // node pair (I, J) with J outside the aggregate
            const int v = (int)vdim;
            for (int64_t k = 0; k < na; k++) {
                const int64_t I = nodes[cnt[a] + k];
                std::vector<int64_t> outside;
                for (int oi = 0; oi < v; oi++) {
                    const int64_t i = I * v + oi;
                    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
                        const int64_t j = col[e], J = j / v, oj = j % v;
                        if (J == I || in_agg(J)) B[(local[J] * v + oj) * s + k * v + oi] += val[e];
                        else outside.push_back(J);
                    }
                }
                std::sort(outside.begin(), outside.end());
                outside.erase(std::unique(outside.begin(), outside.end()), outside.end());
                for (int64_t J : outside) {
                    std::vector<double> M(v * v, 0.0), U;
                    for (int oi = 0; oi < v; oi++) {
                        const int64_t i = I * v + oi;
                        for (int64_t e = rp[i]; e < rp[i + 1]; e++)
                            if (col[e] / v == J) M[oi * v + col[e] % v] -= val[e];
                    }
                    polar_u_s_ut(M, v, U);
                    for (int oi = 0; oi < v; oi++)
                        for (int oj = 0; oj < v; oj++) B[(k * v + oj) * s + k * v + oi] += 0.5 * U[oi * v + oj];
                }
            }
        }
        std::vector<double> Bi;
        if (!spd_inverse(B, s, Bi)) { bad |= 1; continue; }
        std::copy(Bi.begin(), Bi.end(), inv.begin() + ioff[a]);
        for (int64_t k = 0; k < na; k++)
            for (int64_t o = 0; o < vdim; o++) {
                const int64_t p = bptr[a] + k * vdim + o;
                rows[p] = (int32_t)(nodes[cnt[a] + k] * vdim + o);
                blk_of[p] = (int32_t)a;
            }
    }
    FAMG_REQUIRE(!bad, AMG_ERR_NOT_SPD, "a compensated block is not SPD (Cholesky pivot <= 0)");
    // chunks of <= 256 rows made of whole blocks
    std::vector<int32_t> chunk{0};
    for (int64_t a = 0; a < nagg;) {
        int64_t b = a, rowsum = 0;
        while (b < nagg && (b == a || rowsum + (bptr[b + 1] - bptr[b]) <= BLK_CHUNK)) {
            rowsum += bptr[b + 1] - bptr[b];
            b++;
        }
        chunk.push_back((int32_t)bptr[b]);
        a = b;
    }
    // drop empty chunks (aggregates of size 0)
    chunk.erase(std::unique(chunk.begin(), chunk.end()), chunk.end());
    op->nchunks = (int64_t)chunk.size() - 1;
    hipStream_t st = A.ctx->stream;
    op->rows.resize(std::max<int64_t>(1, n));
    op->blk_of.resize(std::max<int64_t>(1, n));
    op->bptr.resize(nagg + 1);
    op->ioff.resize(nagg + 1);
    op->chunk.resize(chunk.size());
    op->inv.resize(std::max<int64_t>(1, ioff[nagg]));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->rows.get(), rows.data(), n * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->blk_of.get(), blk_of.data(), n * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->bptr.get(), bptr.data(), (nagg + 1) * 8, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->ioff.get(), ioff.data(), (nagg + 1) * 8, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->chunk.get(), chunk.data(), chunk.size() * 4, hipMemcpyHostToDevice, st));
    if (ioff[nagg])
        FAMG_CHECK_HIP(hipMemcpyAsync(op->inv.get(), inv.data(), ioff[nagg] * 8, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    op->h_bptr = std::move(bptr);
    op->h_rows = std::move(rows);
    return op;
}

// BlockSmoother::into_sparse_mat (:122-146): the block-diagonal inverse as CSR
CsrPtr block_smoother_to_csr(BlockSmootherOp &B) {
    const int64_t n = B.nrows;
    std::vector<double> inv(B.inv.size());
    FAMG_CHECK_HIP(hipMemcpyAsync(inv.data(), B.inv.get(), inv.size() * 8, hipMemcpyDeviceToHost, B.ctx->stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(B.ctx->stream));
    std::vector<int64_t> cntr(n + 1, 0), ioff(B.nblocks + 1, 0);
    for (int64_t a = 0; a < B.nblocks; a++) {
        const int64_t s = B.h_bptr[a + 1] - B.h_bptr[a];
        ioff[a + 1] = ioff[a] + s * s;
        for (int64_t k = B.h_bptr[a]; k < B.h_bptr[a + 1]; k++) cntr[B.h_rows[k] + 1] = s;
    }
    for (int64_t i = 0; i < n; i++) cntr[i + 1] += cntr[i];
    std::vector<int64_t> col(cntr[n]);
    std::vector<double> val(cntr[n]);
    for (int64_t a = 0; a < B.nblocks; a++) {
        const int64_t b0 = B.h_bptr[a], s = B.h_bptr[a + 1] - b0;
        // rows of a block are ascending in original numbering -> sorted columns
        for (int64_t i = 0; i < s; i++) {
            const int64_t r = B.h_rows[b0 + i];
            for (int64_t j = 0; j < s; j++) {
                col[cntr[r] + j] = B.h_rows[b0 + j];
                val[cntr[r] + j] = inv[ioff[a] + j * s + i];
            }
        }
    }
    auto p = make_csr(B.ctx);
    csr_from_host(p->m, B.ctx, n, n, cntr.data(), col.data(), val.data());
    p->nrows = p->ncols = n;
    return p;
}

}  // namespace famg

extern "C" {

amg_status amg_block_smoother_create(const amg_linop *A, const int64_t *node_partition, int64_t naggregates,
                                     int64_t block_size, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(A && A->op && node_partition && out && naggregates >= 0, AMG_ERR_INVALID, "bad argument");
        auto a = std::dynamic_pointer_cast<CsrOp>(A->op);
        FAMG_REQUIRE(a, AMG_ERR_INVALID, "operator is not a CSR matrix");
        a->ctx->set_device();
        *out = new amg_linop{make_block_smoother(*a, node_partition, naggregates, block_size)};
    });
}

amg_status amg_block_smoother_to_csr(const amg_linop *bs, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(bs && bs->op && out, AMG_ERR_INVALID, "bad argument");
        auto b = std::dynamic_pointer_cast<BlockSmootherOp>(bs->op);
        FAMG_REQUIRE(b, AMG_ERR_INVALID, "operator is not a block smoother");
        b->ctx->set_device();
        *out = new amg_linop{block_smoother_to_csr(*b)};
    });
}

}  // extern "C"
