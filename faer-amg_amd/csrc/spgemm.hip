// spgemm.hip -- Galerkin setup kernels: sparse x sparse, transpose, Jacobi
// smoothing of the tentative interpolation.
//
// Replaces faer's sparse products at interpolation/mod.rs:716-720 (R = P^T,
// A_c = R (A P)), :824-828 and :927-946 (P <- P - omega D^-1 A P).
//
// SpGEMM is row-per-wavefront with an LDS hash table (two phases: symbolic
// row counts -> scan -> numeric).  The numeric phase walks the entries of
// A's row in ascending k and, for each k, spreads B's row over the 64 lanes;
// every C entry therefore accumulates its products in ascending k with fma,
// exactly the order of the CPU oracle, so C is bitwise identical to it.
// Transpose is count -> scan -> atomic scatter -> per-row sort (deterministic
// output because sort keys are distinct).
#include <algorithm>
#include <cmath>

#include "famg.hpp"

namespace famg {

__device__ __forceinline__ unsigned hash32(int32_t j) { return static_cast<unsigned>(j) * 2654435761u; }

// --------------------------------------------------------------- SpGEMM

__global__ void k_spgemm_ub(const int64_t *arp, const int32_t *acol, const int64_t *brp, int64_t m,
                            unsigned long long *maxub) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long s = 0;
    if (i < m)
        for (int64_t e = arp[i]; e < arp[i + 1]; e++) s += brp[acol[e] + 1] - brp[acol[e]];
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(s, off);
        s = s > o ? s : o;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxub, s);
}

// Linear-probing insert; returns 1 if newly inserted, 0 if present, -1 if the
// table is full (only possible in the symbolic pass when the distinct count was
// not bounded in advance).
template <int TBL>
__device__ __forceinline__ int hash_insert(int32_t *keys, int32_t j, int *slot_out) {
    unsigned h = hash32(j) & (TBL - 1);
    for (int probe = 0; probe < TBL; probe++) {
        const int32_t old = atomicCAS(&keys[h], -1, j);
        if (old == -1) { *slot_out = (int)h; return 1; }
        if (old == j) { *slot_out = (int)h; return 0; }
        h = (h + 1) & (TBL - 1);
    }
    return -1;
}

template <int TBL>
__device__ __forceinline__ int hash_find(const int32_t *keys, int32_t j) {
    unsigned h = hash32(j) & (TBL - 1);
    while (keys[h] != j) h = (h + 1) & (TBL - 1);
    return (int)h;
}

template <int TBL>
__global__ __launch_bounds__(64) void k_spgemm_symbolic(const int64_t *arp, const int32_t *acol,
                                                        const int64_t *brp, const int32_t *bcol,
                                                        int64_t m, int64_t *cnt,
                                                        unsigned long long *maxcnt, int *overflow) {
    __shared__ int32_t keys[TBL];
    const int lane = threadIdx.x;
    for (int64_t row = blockIdx.x; row < m; row += gridDim.x) {
        for (int t = lane; t < TBL; t += 64) keys[t] = -1;
        __syncthreads();
        int local = 0, full = 0, slot;
        for (int64_t e = arp[row]; e < arp[row + 1]; e++) {
            const int32_t k = acol[e];
            for (int64_t f = brp[k] + lane; f < brp[k + 1]; f += 64) {
                const int ins = hash_insert<TBL>(keys, bcol[f], &slot);
                if (ins < 0) full = 1;
                else local += ins;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            local += __shfl_xor(local, off);
            full |= __shfl_xor(full, off);
        }
        if (lane == 0) {
            cnt[row] = local;
            atomicMax(maxcnt, (unsigned long long)local);
            if (full || 2 * local > TBL) *overflow = 1;
        }
        __syncthreads();
    }
}

template <int TBL>
__global__ __launch_bounds__(64) void k_spgemm_numeric(const int64_t *arp, const int32_t *acol,
                                                       const double *aval, const int64_t *brp,
                                                       const int32_t *bcol, const double *bval,
                                                       int64_t m, const int64_t *crp, int32_t *ccol,
                                                       double *cval) {
    __shared__ int32_t keys[TBL];
    __shared__ int32_t spos[TBL];
    __shared__ int32_t list[TBL / 2];
    __shared__ double acc[TBL / 2];
    __shared__ int cntsh;
    const int lane = threadIdx.x;
    for (int64_t row = blockIdx.x; row < m; row += gridDim.x) {
        for (int t = lane; t < TBL; t += 64) keys[t] = -1;
        if (lane == 0) cntsh = 0;
        __syncthreads();
        for (int64_t e = arp[row]; e < arp[row + 1]; e++) {
            const int32_t k = acol[e];
            for (int64_t f = brp[k] + lane; f < brp[k + 1]; f += 64) {
                int slot;
                if (hash_insert<TBL>(keys, bcol[f], &slot) == 1) list[atomicAdd(&cntsh, 1)] = bcol[f];
            }
        }
        __syncthreads();
        const int c = cntsh;
        const int64_t base = crp[row];
        // rank sort of the distinct columns
        for (int u = lane; u < c; u += 64) {
            const int32_t key = list[u];
            int r = 0;
            for (int v = 0; v < c; v++) r += list[v] < key;
            ccol[base + r] = key;
            spos[hash_find<TBL>(keys, key)] = r;
            acc[u] = 0.0;
        }
        __syncthreads();
        for (int64_t e = arp[row]; e < arp[row + 1]; e++) {
            const int32_t k = acol[e];
            const double a = aval[e];
            for (int64_t f = brp[k] + lane; f < brp[k + 1]; f += 64) {
                const int p = spos[hash_find<TBL>(keys, bcol[f])];
                acc[p] = fma(a, bval[f], acc[p]);
            }
            __syncthreads();
        }
        for (int p = lane; p < c; p += 64) cval[base + p] = acc[p];
        __syncthreads();
    }
}

static unsigned spgemm_grid(int64_t m) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(m, 256 * 16));
}

// symbolic pass with a TBL-entry table: per-row distinct counts; returns the
// max count, or -1 if some row did not fit (count > TBL/2)
template <int TBL>
static int64_t spgemm_symbolic(const GpuCsr &A, const GpuCsr &B, int64_t *cnt, Ctx &ctx) {
    const int64_t m = A.nrows;
    hipStream_t s = ctx.stream;
    DevBuf<unsigned long long> mx(1);
    DevBuf<int> of(1);
    FAMG_CHECK_HIP(hipMemsetAsync(mx.get(), 0, sizeof(unsigned long long), s));
    FAMG_CHECK_HIP(hipMemsetAsync(of.get(), 0, sizeof(int), s));
    if (m)
        hipLaunchKernelGGL(k_spgemm_symbolic<TBL>, dim3(spgemm_grid(m)), dim3(64), 0, s,
                           A.rp64.get(), A.col.get(), B.rp64.get(), B.col.get(), m, cnt, mx.get(),
                           of.get());
    FAMG_CHECK_HIP(hipGetLastError());
    unsigned long long hmx = 0;
    int hof = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&hmx, mx.get(), sizeof(hmx), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(&hof, of.get(), sizeof(hof), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return hof ? -1 : (int64_t)hmx;
}

template <int TBL>
static void spgemm_numeric(const GpuCsr &A, const GpuCsr &B, GpuCsr &C, Ctx &ctx) {
    const int64_t m = A.nrows;
    if (m)
        hipLaunchKernelGGL(k_spgemm_numeric<TBL>, dim3(spgemm_grid(m)), dim3(64), 0, ctx.stream,
                           A.rp64.get(), A.col.get(), A.val.get(), B.rp64.get(), B.col.get(),
                           B.val.get(), m, C.rp64.get(), C.col.get(), C.val.get());
    FAMG_CHECK_HIP(hipGetLastError());
}

void spgemm(const GpuCsr &A, const GpuCsr &B, GpuCsr &C, bool finalize) {
    FAMG_REQUIRE(A.ncols == B.nrows, AMG_ERR_DIM, "spgemm: A.ncols != B.nrows");
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    DevBuf<unsigned long long> mx(1);
    FAMG_CHECK_HIP(hipMemsetAsync(mx.get(), 0, sizeof(unsigned long long), s));
    if (A.nrows)
        hipLaunchKernelGGL(k_spgemm_ub, dim3((unsigned)ceil_div(A.nrows, 256)), dim3(256), 0, s,
                           A.rp64.get(), A.col.get(), B.rp64.get(), A.nrows, mx.get());
    unsigned long long maxub = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&maxub, mx.get(), sizeof(maxub), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    // symbolic table: sized from the product bound when it is small, otherwise
    // the largest table with overflow detection; numeric table: from the true
    // per-row maximum of distinct columns.
    const int64_t bound = std::min<int64_t>((int64_t)maxub, B.ncols);
    const int64_t m = A.nrows;
    DevBuf<int64_t> cnt(m + 1);
    int64_t maxc;
    if (bound <= 32) maxc = spgemm_symbolic<64>(A, B, cnt.get(), ctx);
    else if (bound <= 128) maxc = spgemm_symbolic<256>(A, B, cnt.get(), ctx);
    else if (bound <= 512) maxc = spgemm_symbolic<1024>(A, B, cnt.get(), ctx);
    else maxc = spgemm_symbolic<8192>(A, B, cnt.get(), ctx);
    FAMG_REQUIRE(maxc >= 0, AMG_ERR_UNSUPPORTED, "spgemm: a product row exceeds 4096 distinct columns");
    DevBuf<int64_t> rp(m + 1);
    const int64_t nnz = scan_counts(cnt.get(), rp.get(), m, ctx);
    csr_alloc(C, &ctx, m, B.ncols, nnz);
    C.rp64 = std::move(rp);
    if (maxc <= 32) spgemm_numeric<64>(A, B, C, ctx);
    else if (maxc <= 128) spgemm_numeric<256>(A, B, C, ctx);
    else if (maxc <= 512) spgemm_numeric<1024>(A, B, C, ctx);
    else if (maxc <= 2048) spgemm_numeric<4096>(A, B, C, ctx);
    else spgemm_numeric<8192>(A, B, C, ctx);
    if (finalize) csr_finalize(C);
}

// ------------------------------------------------------------- transpose

__global__ void k_t_count(const int32_t *col, int64_t nnz, unsigned long long *cnt) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < nnz) atomicAdd(&cnt[col[e]], 1ull);
}

__global__ void k_t_fill(const int64_t *rp, const int32_t *col, const double *val, int64_t m,
                         unsigned long long *pos, int32_t *tcol, double *tval) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        const unsigned long long p = atomicAdd(&pos[col[e]], 1ull);
        tcol[p] = static_cast<int32_t>(i);
        tval[p] = val[e];
    }
}

// per-row sort by column (workgroup per row): rank sort of distinct keys in
// LDS; rows longer than TSORT_CAP fall back to a serial insertion sort
template <int TSORT_CAP, int TSORT_BS>
__global__ __launch_bounds__(TSORT_BS) void k_row_sort(const int64_t *rp, int64_t m, int32_t *col, double *val) {
    __shared__ int32_t sk[TSORT_CAP];
    __shared__ double sv[TSORT_CAP];
    const int lane = threadIdx.x;
    for (int64_t row = blockIdx.x; row < m; row += gridDim.x) {
        const int64_t s0 = rp[row], len = rp[row + 1] - s0;
        if (len <= 1) continue;
        if (len <= TSORT_CAP) {
            for (int u = lane; u < len; u += TSORT_BS) { sk[u] = col[s0 + u]; sv[u] = val[s0 + u]; }
            __syncthreads();
            for (int u = lane; u < len; u += TSORT_BS) {
                const int32_t key = sk[u];
                int r = 0;
                for (int v = 0; v < len; v++) r += sk[v] < key;
                col[s0 + r] = key;
                val[s0 + r] = sv[u];
            }
            __syncthreads();
        } else if (lane == 0) {
            for (int64_t a = 1; a < len; a++) {
                const int32_t k = col[s0 + a];
                const double v = val[s0 + a];
                int64_t b = a - 1;
                while (b >= 0 && col[s0 + b] > k) { col[s0 + b + 1] = col[s0 + b]; val[s0 + b + 1] = val[s0 + b]; b--; }
                col[s0 + b + 1] = k;
                val[s0 + b + 1] = v;
            }
        }
    }
}

__global__ void k_max_len(const int64_t *rp, int64_t n, unsigned long long *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long v = i < n ? (unsigned long long)(rp[i + 1] - rp[i]) : 0ull;
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = v > o ? v : o;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, v);
}

void transpose(const GpuCsr &A, GpuCsr &T) {
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    const int64_t n = A.ncols;
    DevBuf<unsigned long long> cnt(n + 1);
    FAMG_CHECK_HIP(hipMemsetAsync(cnt.get(), 0, (n + 1) * sizeof(unsigned long long), s));
    if (A.nnz)
        hipLaunchKernelGGL(k_t_count, dim3((unsigned)ceil_div(A.nnz, 256)), dim3(256), 0, s,
                           A.col.get(), A.nnz, cnt.get());
    DevBuf<int64_t> rp(n + 1);
    const int64_t nnz = scan_counts(reinterpret_cast<const int64_t *>(cnt.get()), rp.get(), n, ctx);
    FAMG_REQUIRE(nnz == A.nnz, AMG_ERR_INVALID, "transpose: count mismatch");
    csr_alloc(T, &ctx, n, A.nrows, nnz);
    T.rp64 = std::move(rp);
    FAMG_CHECK_HIP(hipMemcpyAsync(cnt.get(), T.rp64.get(), n * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    FAMG_CHECK_HIP(hipMemsetAsync(cnt.get() + n, 0, sizeof(unsigned long long), s));
    if (A.nrows)
        hipLaunchKernelGGL(k_t_fill, dim3((unsigned)ceil_div(A.nrows, 256)), dim3(256), 0, s,
                           A.rp64.get(), A.col.get(), A.val.get(), A.nrows, cnt.get(), T.col.get(),
                           T.val.get());
    if (n) {
        hipLaunchKernelGGL(k_max_len, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                           T.rp64.get(), n, cnt.get() + n);
        unsigned long long maxlen = 0;
        FAMG_CHECK_HIP(hipMemcpyAsync(&maxlen, cnt.get() + n, sizeof(maxlen), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        const unsigned g = (unsigned)std::min<int64_t>(n, 4096);
        if (maxlen <= 2048)
            hipLaunchKernelGGL((k_row_sort<2048, 64>), dim3(g), dim3(64), 0, s, T.rp64.get(), n,
                               T.col.get(), T.val.get());
        else
            hipLaunchKernelGGL((k_row_sort<8192, 256>), dim3(g), dim3(256), 0, s, T.rp64.get(), n,
                               T.col.get(), T.val.get());
    }
    FAMG_CHECK_HIP(hipGetLastError());
    csr_finalize(T);
}

// ------------------------------------------------- interpolation smoothing

// S = A P already computed; S_i* *= -(omega * (1/a_ii)); S += P on P's pattern
// (interpolation/mod.rs:932-945).  bad -> 1 if a diagonal is <= 1e-6 or P's
// pattern is not contained in S's.
__global__ void k_smooth_fix(const int64_t *srp, const int32_t *scol, double *sval,
                             const int64_t *prp, const int32_t *pcol, const double *pval,
                             const double *diag, double omega, int64_t m, int *bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const double aii = diag[i];
    if (!(aii > 1e-6)) { *bad = 1; return; }
    const double scalar = omega * (1.0 / aii);
    const int64_t s0 = srp[i], s1 = srp[i + 1];
    for (int64_t e = s0; e < s1; e++) sval[e] = sval[e] * -scalar;
    for (int64_t e = prp[i]; e < prp[i + 1]; e++) {
        int64_t lo = s0, hi = s1;
        const int32_t j = pcol[e];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (scol[mid] < j) lo = mid + 1;
            else hi = mid;
        }
        if (lo >= s1 || scol[lo] != j) { *bad = 2; return; }
        sval[lo] = sval[lo] + pval[e];
    }
}

void smooth_interp_fixup(GpuCsr &S, const GpuCsr &P, const double *diag, double omega) {
    Ctx &ctx = *S.ctx;
    hipStream_t s = ctx.stream;
    DevBuf<int> bad(1);
    FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
    if (S.nrows)
        hipLaunchKernelGGL(k_smooth_fix, dim3((unsigned)ceil_div(S.nrows, 256)), dim3(256), 0, s,
                           S.rp64.get(), S.col.get(), S.val.get(), P.rp64.get(), P.col.get(),
                           P.val.get(), diag, omega, S.nrows, bad.get());
    int h = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&h, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    FAMG_REQUIRE(h != 1, AMG_ERR_INVALID, "smooth_interpolation: diagonal nearly zero");
    FAMG_REQUIRE(h != 2, AMG_ERR_INVALID, "smooth_interpolation: P pattern not within A*P");
    // the values changed in place: rebuild the derived SpMV storage (SELL copy)
    csr_finalize(S);
}

}  // namespace famg
