// chol.hip -- the coarsest-level Cholesky solve at any size
// (SparseCholeskySolve, coarse_solvers.rs:164-206: faer's sparse LLt of the
// coarsest operator, whatever its size -- HierarchyConfig.max_levels,
// hierarchy.rs:25, and a coarsening that stalls both leave large coarsest levels).
//
// Up to 8192 rows the coarse solve is one GEMV with the explicit inverse
// (ops.hip).  Above that a dense inverse stops being an option (n^2 doubles,
// n^3 host work), so:
//   setup (host): reverse Cuthill-McKee order p, the envelope (profile) Cholesky
//     factor of P A P^T (row i spans columns fc[i] .. i, fill stays inside the
//     envelope), cut into 64-row blocks: block k = the dense slab of its rows over
//     columns [cmin_k, k0) (column-major, zeros left of a row's envelope) plus
//     the explicit inverse M_k of its 64 x 64 lower-triangular diagonal block;
//   apply (device, one 1024-thread workgroup, one launch): z = P b; forward
//     z_k = M_k (z_k - S_k z[cmin_k, k0)) block by block; backward right-looking
//     x_k = M_k^T z_k, then z[cmin_k, k0) -= S_k^T x_k; out = P^T x.
// Every partial sum runs in a fixed order (deterministic); the result agrees with
// the oracle's envelope factor (same LLt, another numbering) to rounding.
#include <algorithm>
#include <cmath>

#include "famg.hpp"

namespace famg {

constexpr int CB = 64;  // rows per block

struct CholEnvArgs {
    const double *slab;     // per block: w_k x 64 column-major
    const int64_t *soff;    // per block: slab offset
    const int32_t *cmin;    // per block: first column of the slab
    const double *mc;       // per block: M_k column-major (64 x 64)
    const double *mr;       // per block: M_k^T column-major (= M_k row-major)
    const int32_t *perm;    // new -> old
    int64_t n, nb;
    const double *b;
    double *out, *z;        // z: nb * 64 scratch
};

__global__ __launch_bounds__(1024) void k_chol_env(CholEnvArgs a) {
    __shared__ double part[16][CB];
    __shared__ double tv[CB];
    const int tid = threadIdx.x, r = tid & 63, q = tid >> 6;
    for (int64_t i = tid; i < a.nb * CB; i += 1024) a.z[i] = i < a.n ? a.b[a.perm[i]] : 0.0;
    __threadfence_block();
    __syncthreads();
    // forward: L y = P b
    for (int64_t k = 0; k < a.nb; k++) {
        const int64_t k0 = k * CB;
        const int32_t cm = a.cmin[k];
        const int64_t w = k0 - cm;
        const double *S = a.slab + a.soff[k];
        double acc = 0.0;
        for (int64_t c = q; c < w; c += 16) acc = fma(S[c * CB + r], a.z[cm + c], acc);
        part[q][r] = acc;
        __syncthreads();
        if (q == 0) {
            double t = a.z[k0 + r];
#pragma unroll
            for (int j = 0; j < 16; j++) t -= part[j][r];
            tv[r] = t;
        }
        __syncthreads();
        if (q == 0) {
            const double *M = a.mc + k * CB * CB;
            double y = 0.0;
            for (int c = 0; c <= r; c++) y = fma(M[c * CB + r], tv[c], y);
            a.z[k0 + r] = y;
        }
        __threadfence_block();
        __syncthreads();
    }
    // backward: L^T x = y, right-looking
    for (int64_t k = a.nb - 1; k >= 0; k--) {
        const int64_t k0 = k * CB;
        const int32_t cm = a.cmin[k];
        const int64_t w = k0 - cm;
        if (q == 0) {
            const double *M = a.mr + k * CB * CB;
            double x = 0.0;
            for (int c = r; c < CB; c++) x = fma(M[c * CB + r], a.z[k0 + c], x);
            tv[r] = x;
        }
        __syncthreads();
        if (q == 0) a.z[k0 + r] = tv[r];
        const double xr = tv[r];
        const double *S = a.slab + a.soff[k];
        for (int64_t c = q; c < w; c += 16) {  // one wave per column: a fixed butterfly sum
            double v = S[c * CB + r] * xr;
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if (r == 0) a.z[cm + c] -= v;
        }
        __threadfence_block();
        __syncthreads();
    }
    for (int64_t i = tid; i < a.n; i += 1024) a.out[a.perm[i]] = a.z[i];
}

std::shared_ptr<CoarseCholOp> make_coarse_chol_env(CsrOp &A) {
    const int64_t n = A.nrows;
    FAMG_REQUIRE(n < (int64_t(1) << 31), AMG_ERR_UNSUPPORTED, "coarse Cholesky: more than 2^31 rows");
    std::vector<int64_t> rp(n + 1), col64(A.m.nnz);
    std::vector<double> val(A.m.nnz);
    csr_to_host(A.m, rp.data(), col64.data(), val.data());
    std::vector<int32_t> col(col64.begin(), col64.end());
    const std::vector<int32_t> p = rcm_order(rp, col, n, 1);  // new -> old
    std::vector<int32_t> q(n);
    for (int64_t i = 0; i < n; i++) q[p[i]] = (int32_t)i;
    // envelope of the lower triangle of P A P^T
    std::vector<int64_t> fc(n), ep(n + 1, 0);
    for (int64_t i = 0; i < n; i++) {
        int64_t f = i;
        const int64_t r = p[i];
        for (int64_t e = rp[r]; e < rp[r + 1]; e++) f = std::min<int64_t>(f, q[col[e]]);
        fc[i] = f;
        ep[i + 1] = ep[i] + (i - f + 1);
    }
    std::vector<double> L(ep[n], 0.0);
    for (int64_t i = 0; i < n; i++) {
        const int64_t r = p[i];
        for (int64_t e = rp[r]; e < rp[r + 1]; e++) {
            const int64_t j = q[col[e]];
            if (j <= i) L[ep[i] + j - fc[i]] += val[e];
        }
    }
    for (int64_t i = 0; i < n; i++) {
        double *li = L.data() + ep[i] - fc[i];
        for (int64_t j = fc[i]; j < i; j++) {
            const double *lj = L.data() + ep[j] - fc[j];
            double t = li[j];
            for (int64_t k = std::max(fc[i], fc[j]); k < j; k++) t -= li[k] * lj[k];
            li[j] = t / lj[j];
        }
        double d = li[i];
        for (int64_t k = fc[i]; k < i; k++) d -= li[k] * li[k];
        FAMG_REQUIRE(d > 0.0, AMG_ERR_NOT_SPD, "coarse matrix is not SPD (Cholesky pivot <= 0)");
        li[i] = std::sqrt(d);
    }
    // 64-row blocks: off-diagonal slabs (column-major) and the inverses of the diagonal blocks
    const int64_t nb = ceil_div(n, CB);
    std::vector<int32_t> cmin(nb);
    std::vector<int64_t> soff(nb + 1, 0);
    for (int64_t k = 0; k < nb; k++) {
        const int64_t k0 = k * CB, k1 = std::min(n, k0 + CB);
        int64_t c = k0;
        for (int64_t i = k0; i < k1; i++) c = std::min(c, fc[i]);
        cmin[k] = (int32_t)c;
        soff[k + 1] = soff[k] + (k0 - c) * CB;
    }
    std::vector<double> slab(std::max<int64_t>(1, soff[nb]), 0.0), mc(nb * CB * CB, 0.0), mr(nb * CB * CB, 0.0);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t k = 0; k < nb; k++) {
        const int64_t k0 = k * CB, k1 = std::min(n, k0 + CB), cm = cmin[k];
        for (int64_t i = k0; i < k1; i++)
            for (int64_t j = std::max(fc[i], cm); j < k0; j++) slab[soff[k] + (j - cm) * CB + (i - k0)] = L[ep[i] + j - fc[i]];
        // D = the diagonal block (identity past n); M = D^-1 by forward substitution
        double D[CB][CB] = {}, M[CB][CB] = {};
        for (int i = 0; i < CB; i++) {
            if (k0 + i >= n) { D[i][i] = 1.0; continue; }
            for (int64_t j = std::max(fc[k0 + i], k0); j <= k0 + i; j++) D[i][j - k0] = L[ep[k0 + i] + j - fc[k0 + i]];
        }
        for (int c = 0; c < CB; c++)
            for (int i = c; i < CB; i++) {
                double t = i == c ? 1.0 : 0.0;
                for (int j = c; j < i; j++) t -= D[i][j] * M[j][c];
                M[i][c] = t / D[i][i];
            }
        for (int i = 0; i < CB; i++)
            for (int c = 0; c < CB; c++) {
                mc[k * CB * CB + c * CB + i] = M[i][c];  // column-major M
                mr[k * CB * CB + c * CB + i] = M[c][i];  // column-major M^T
            }
    }
    auto op = std::make_shared<CoarseCholOp>();
    op->ctx = A.ctx;
    op->nrows = op->ncols = n;
    op->nb = nb;
    op->env_bytes = (int64_t)slab.size() * 8;
    hipStream_t s = A.ctx->stream;
    op->slab.resize(slab.size());
    op->soff.resize(nb + 1);
    op->cmin.resize(nb);
    op->mc.resize(mc.size());
    op->mr.resize(mr.size());
    op->perm.resize(n);
    op->z.resize(nb * CB);
    FAMG_CHECK_HIP(hipMemcpyAsync(op->slab.get(), slab.data(), slab.size() * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->soff.get(), soff.data(), (nb + 1) * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->cmin.get(), cmin.data(), nb * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->mc.get(), mc.data(), mc.size() * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->mr.get(), mr.data(), mr.size() * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(op->perm.get(), p.data(), n * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return op;
}

void chol_env_apply(const CoarseCholOp &op, double *out, const double *rhs, hipStream_t s) {
    CholEnvArgs a{};
    a.slab = op.slab.get();
    a.soff = op.soff.get();
    a.cmin = op.cmin.get();
    a.mc = op.mc.get();
    a.mr = op.mr.get();
    a.perm = op.perm.get();
    a.n = op.nrows;
    a.nb = op.nb;
    a.b = rhs;
    a.out = out;
    a.z = const_cast<double *>(op.z.get());
    log_launch("chol-env", -1, -1, op.nrows, 2 * op.env_bytes + 4 * op.nb * CB * CB * 8 + 28 * op.nrows);
    k_chol_env<<<dim3(1), dim3(1024), 0, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
