// bsr.hip -- 3x3 block storage (node-row SELL) for the SpMV of block
// operators: vector problems with 3 dofs per node interleaved, the layout of
// the reference's SparseMatOp block_size = 3 (core.rs:12-17) -- Flan_1565
// (config C5), the in-tree Q1-elasticity stand-in, and every operator the SA
// setup derives from them (P, R = P^T, A_c = R A P with 3 candidates per
// aggregate are 3x3-blocked too).
//
// A scalar CSR/SELL entry of such a matrix costs 12 B (8 value + 4 column) and
// one x gather; a 3x3 block carries 9 values under one node column (76 B per
// 9 entries = 8.4 B/entry) and its three x operands are adjacent.  Layout:
// slices of 64 node rows (3 dof rows each, one lane per node row), w_s block
// steps per slice (the slice's longest node row; padding blocks have value
// 0.0 at an in-range column).  Step t of a slice is one 4864-B unit:
//   [4 x 1024 B: value pairs (k, k+1), k = 0, 2, 4, 6 | 512 B: value k = 8 |
//    256 B: node column J]        (value k of a block = a(3I + k/3, 3J + k%3))
// so each lane reads 16-B, 16-B, 16-B, 16-B, 8-B and 4-B coalesced units.
// Dof row 3I + r sums its blocks in ascending J and c = 0, 1, 2 with fma --
// its stored (ascending column) order -- so results are bitwise those of the
// CSR / SELL kernels (missing entries of a block add exact zeros).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "famg.hpp"

namespace famg {

typedef double bsr_dbl2_t __attribute__((ext_vector_type(2)));

constexpr int BSR_B = 3;
constexpr int BSR_C = 64;                                   // node rows per slice
constexpr int64_t BSR_STEP = BSR_C * (9 * 8 + 4);           // 4864 B per block step
constexpr int BSR_K8 = 4 * BSR_C * 16;                      // offset of value 8
constexpr int BSR_COL = BSR_K8 + BSR_C * 8;                 // offset of the node columns

struct BsrEpi {
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
    double *y2;  // SETDF: d * y beside y (the next level's first Jacobi step from zero)
};

struct BsrArgs {
    const char *data;
    const int32_t *row0;  // node-row start per slice (+1)
    const int32_t *soff;  // step offset per slice (+1)
    int32_t slice0, nslices;
    BsrEpi e;
    int32_t jmask;  // node column mask: -1; 0 = measurement only (FAMG_BSR_DIAG=1: every x gather at node 0)
};

template <int MODE> struct BsrRow {
    double xr = 0.0, br = 0.0, dr = 0.0, yr = 0.0;
    __device__ __forceinline__ void load(const BsrEpi &a, int i) {
        if constexpr (MODE == SPMV_JACOBI) {
            xr = a.x[i];
            br = a.b[i];
            dr = a.dc ? a.dt[a.dc[i]] : a.d[i];
        }
        if constexpr (MODE == SPMV_RESID) br = a.b[i];
        if constexpr (MODE == SPMV_ADD) yr = a.y[i];
        if constexpr (MODE == SPMV_SETDF) dr = a.dc ? a.dt[a.dc[i]] : a.d[i];
    }
    __device__ __forceinline__ void store(const BsrEpi &a, int i, double acc) const {
        if constexpr (MODE == SPMV_SET) a.y[i] = acc;
        else if constexpr (MODE == SPMV_SETDF) {
            a.y[i] = acc;
            a.y2[i] = dr * acc;  // vec_mul(_coded)'s product
        } else if constexpr (MODE == SPMV_ADD) a.y[i] = yr + acc;
        else if constexpr (MODE == SPMV_RESID) a.y[i] = br - acc;
        else a.y[i] = xr + dr * (br - acc);  // JACOBI
    }
};

// U block steps: every load of the group is issued before the fmas
template <int U>
__device__ __forceinline__ void bsr_steps(const char *__restrict__ st, int lane, const double *__restrict__ x,
                                          double &a0, double &a1, double &a2, int jmask) {
    double v[U][9], xx[U][3];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const char *p = st + (int64_t)u * BSR_STEP;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bsr_dbl2_t w = __builtin_nontemporal_load(reinterpret_cast<const bsr_dbl2_t *>(p + q * 1024) + lane);
            v[u][2 * q] = w.x;
            v[u][2 * q + 1] = w.y;
        }
        v[u][8] = __builtin_nontemporal_load(reinterpret_cast<const double *>(p + BSR_K8) + lane);
        const int J = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(p + BSR_COL) + lane) & jmask;
        const double *xp = x + 3 * (int64_t)J;
        xx[u][0] = xp[0];
        xx[u][1] = xp[1];
        xx[u][2] = xp[2];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        a0 = fma(v[u][0], xx[u][0], a0);
        a0 = fma(v[u][1], xx[u][1], a0);
        a0 = fma(v[u][2], xx[u][2], a0);
        a1 = fma(v[u][3], xx[u][0], a1);
        a1 = fma(v[u][4], xx[u][1], a1);
        a1 = fma(v[u][5], xx[u][2], a1);
        a2 = fma(v[u][6], xx[u][0], a2);
        a2 = fma(v[u][7], xx[u][1], a2);
        a2 = fma(v[u][8], xx[u][2], a2);
    }
}

// WPB waves (slices) per workgroup: 4, or 1 for a matrix of few slices, so that
// its few hundred waves spread over every CU (625 slices in 4-wave workgroups
// left 99 of the 256 CUs idle: C5's R_0 / A_1)
template <int MODE, int WPB>
__global__ __launch_bounds__(256) void spmv_bsr3_kernel(BsrArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = __builtin_amdgcn_readfirstlane(blk * WPB + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int s = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int I = a.row0[s] + lane;
    const bool live = I < a.row0[s + 1];
    BsrRow<MODE> r0, r1, r2;
    if (live) {
        r0.load(a.e, 3 * I);
        r1.load(a.e, 3 * I + 1);
        r2.load(a.e, 3 * I + 2);
    }
    const int t0 = a.soff[s], w = a.soff[s + 1] - t0;
    const char *st = a.data + (int64_t)t0 * BSR_STEP;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    int t = 0;
    for (; t + 4 <= w; t += 4) bsr_steps<4>(st + (int64_t)t * BSR_STEP, lane, a.e.x, a0, a1, a2, a.jmask);
    switch (w - t) {
    case 1: bsr_steps<1>(st + (int64_t)t * BSR_STEP, lane, a.e.x, a0, a1, a2, a.jmask); break;
    case 2: bsr_steps<2>(st + (int64_t)t * BSR_STEP, lane, a.e.x, a0, a1, a2, a.jmask); break;
    case 3: bsr_steps<3>(st + (int64_t)t * BSR_STEP, lane, a.e.x, a0, a1, a2, a.jmask); break;
    default: break;
    }
    if (live) {
        r0.store(a.e, 3 * I, a0);
        r1.store(a.e, 3 * I + 1, a1);
        r2.store(a.e, 3 * I + 2, a2);
    }
}

// ------------------------------------------------------------ columns-first form
// The kernel above waits two dependent round trips per group of block steps (the
// node columns, then the x operands they address).  Here (FLAG_BSR_KERNEL >= 1,
// slices of <= BSR_PCOL steps) a wave first loads the node columns of all its
// slice's steps (one round trip; a step past the slice's width reloads the last
// one), then walks U-step batches whose value and x loads are independent of
// each other -- one round trip per batch -- and with PIPE issues batch b + 1
// before summing batch b.  Same fma order per dof row: bitwise the kernel above.
constexpr int BSR_PCOL = 32;

template <int U>
__device__ __forceinline__ void bsr_issue(const char *__restrict__ st, int lane, const double *__restrict__ x,
                                          const int32_t *J, int b, int tl, double (&v)[U][9], double (&xx)[U][3]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        const char *p = st + (int64_t)min(b * U + u, tl) * BSR_STEP;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bsr_dbl2_t w = __builtin_nontemporal_load(reinterpret_cast<const bsr_dbl2_t *>(p + q * 1024) + lane);
            v[u][2 * q] = w.x;
            v[u][2 * q + 1] = w.y;
        }
        v[u][8] = __builtin_nontemporal_load(reinterpret_cast<const double *>(p + BSR_K8) + lane);
        const double *xp = x + 3 * (int64_t)J[b * U + u];
        xx[u][0] = xp[0];
        xx[u][1] = xp[1];
        xx[u][2] = xp[2];
    }
}

template <int U>
__device__ __forceinline__ void bsr_sum(const double (&v)[U][9], const double (&xx)[U][3], int b, int w, double &a0,
                                        double &a1, double &a2) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (b * U + u >= w) break;  // clamped steps past the slice's width: loaded, never summed
        a0 = fma(v[u][0], xx[u][0], a0);
        a0 = fma(v[u][1], xx[u][1], a0);
        a0 = fma(v[u][2], xx[u][2], a0);
        a1 = fma(v[u][3], xx[u][0], a1);
        a1 = fma(v[u][4], xx[u][1], a1);
        a1 = fma(v[u][5], xx[u][2], a1);
        a2 = fma(v[u][6], xx[u][0], a2);
        a2 = fma(v[u][7], xx[u][1], a2);
        a2 = fma(v[u][8], xx[u][2], a2);
    }
}

template <int MODE, int U, bool PIPE>
__global__ __launch_bounds__(256) void spmv_bsr3p_kernel(BsrArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int s = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int I = a.row0[s] + lane;
    const bool live = I < a.row0[s + 1];
    const int t0 = a.soff[s], w = a.soff[s + 1] - t0;
    const char *st = a.data + (int64_t)t0 * BSR_STEP;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    BsrRow<MODE> r0, r1, r2;
    if (w > 0) {
        const int tl = w - 1;
        int32_t J[BSR_PCOL];
#pragma unroll
        for (int t = 0; t < BSR_PCOL; t++)
            J[t] = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(st + (int64_t)min(t, tl) * BSR_STEP + BSR_COL) + lane);
        if (live) {
            r0.load(a.e, 3 * I);
            r1.load(a.e, 3 * I + 1);
            r2.load(a.e, 3 * I + 2);
        }
        constexpr int NB = BSR_PCOL / U;
        if constexpr (PIPE) {
            double v0[U][9], x0[U][3], v1[U][9], x1[U][3];
            bsr_issue<U>(st, lane, a.e.x, J, 0, tl, v0, x0);
#pragma unroll
            for (int b = 0; b < NB; b += 2) {
                if (b * U >= w) break;
                if ((b + 1) * U < w) bsr_issue<U>(st, lane, a.e.x, J, b + 1, tl, v1, x1);
                bsr_sum<U>(v0, x0, b, w, a0, a1, a2);
                if ((b + 1) * U >= w) break;
                if ((b + 2) * U < w && b + 2 < NB) bsr_issue<U>(st, lane, a.e.x, J, b + 2, tl, v0, x0);
                bsr_sum<U>(v1, x1, b + 1, w, a0, a1, a2);
            }
        } else {
#pragma unroll
            for (int b = 0; b < NB; b++) {
                if (b * U >= w) break;
                double v[U][9], xx[U][3];
                bsr_issue<U>(st, lane, a.e.x, J, b, tl, v, xx);
                bsr_sum<U>(v, xx, b, w, a0, a1, a2);
            }
        }
    } else if (live) {
        r0.load(a.e, 3 * I);
        r1.load(a.e, 3 * I + 1);
        r2.load(a.e, 3 * I + 2);
    }
    if (live) {
        r0.store(a.e, 3 * I, a0);
        r1.store(a.e, 3 * I + 1, a1);
        r2.store(a.e, 3 * I + 2, a2);
    }
}

// ------------------------------------------------------------ long-row form
// A matrix of few, long node rows (R_0 and A_1 of C5: 625 slices of ~128 block
// steps) is bound by each wave's chain of dependent round trips (node columns,
// then the x operands they address, per group of steps), not by HBM.  Here
// (FLAG_BSR_LONG: slices averaging at least that many steps) a wave walks
// 8-step groups and loads the next group's node columns while the current
// group's values and x operands are in flight: one round trip per 8 steps.
// Two column buffers alternate (no loop-carried copies).  Same fma order per
// dof row: bitwise the kernels above.
constexpr int BSR_LU = 8;
constexpr int64_t BSR_ONE_WAVE_SLICES = 4096;

__device__ __forceinline__ void bsr_long_cols(const char *__restrict__ st, int lane, int g, int tl, int (&J)[BSR_LU]) {
#pragma unroll
    for (int u = 0; u < BSR_LU; u++)  // (the mask is applied at use: no wait on these loads here)
        J[u] = __builtin_nontemporal_load(
            reinterpret_cast<const int32_t *>(st + (int64_t)min(g * BSR_LU + u, tl) * BSR_STEP + BSR_COL) + lane);
}

__device__ __forceinline__ void bsr_long_issue(const char *__restrict__ st, int lane, const double *__restrict__ x,
                                               const int (&J)[BSR_LU], int jmask, int g, int tl,
                                               double (&v)[BSR_LU][9], double (&xx)[BSR_LU][3]) {
#pragma unroll
    for (int u = 0; u < BSR_LU; u++) {
        const char *p = st + (int64_t)min(g * BSR_LU + u, tl) * BSR_STEP;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bsr_dbl2_t w = __builtin_nontemporal_load(reinterpret_cast<const bsr_dbl2_t *>(p + q * 1024) + lane);
            v[u][2 * q] = w.x;
            v[u][2 * q + 1] = w.y;
        }
        v[u][8] = __builtin_nontemporal_load(reinterpret_cast<const double *>(p + BSR_K8) + lane);
        const double *xp = x + 3 * (int64_t)(J[u] & jmask);
        xx[u][0] = xp[0];
        xx[u][1] = xp[1];
        xx[u][2] = xp[2];
    }
}

template <int MODE, int WPB>
__global__ __launch_bounds__(256) void spmv_bsr3l_kernel(BsrArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = __builtin_amdgcn_readfirstlane(blk * WPB + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int s = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int I = a.row0[s] + lane;
    const bool live = I < a.row0[s + 1];
    const int t0 = a.soff[s], w = a.soff[s + 1] - t0;
    const char *st = a.data + (int64_t)t0 * BSR_STEP;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    BsrRow<MODE> r0, r1, r2;
    if (live) {
        r0.load(a.e, 3 * I);
        r1.load(a.e, 3 * I + 1);
        r2.load(a.e, 3 * I + 2);
    }
    if (w > 0) {
        const int tl = w - 1;
        int JA[BSR_LU], JB[BSR_LU];
        bsr_long_cols(st, lane, 0, tl, JA);
        for (int g = 0; g * BSR_LU < w; g += 2) {
            double v[BSR_LU][9], xx[BSR_LU][3];
            bsr_long_issue(st, lane, a.e.x, JA, a.jmask, g, tl, v, xx);
            if ((g + 1) * BSR_LU < w) bsr_long_cols(st, lane, g + 1, tl, JB);
            bsr_sum<BSR_LU>(v, xx, g, w, a0, a1, a2);
            if ((g + 1) * BSR_LU >= w) break;
            bsr_long_issue(st, lane, a.e.x, JB, a.jmask, g + 1, tl, v, xx);
            if ((g + 2) * BSR_LU < w) bsr_long_cols(st, lane, g + 2, tl, JA);
            bsr_sum<BSR_LU>(v, xx, g + 1, w, a0, a1, a2);
        }
    }
    if (live) {
        r0.store(a.e, 3 * I, a0);
        r1.store(a.e, 3 * I + 1, a1);
        r2.store(a.e, 3 * I + 2, a2);
    }
}

static bool bsr_disabled() {
    static const bool off = [] {
        const char *e = getenv("FAMG_NO_BSR");
        return e && e[0] == '1';
    }();
    return off;
}

// Build the block storage when the matrix is 3x3-blocked (rows 3I..3I+2 share
// their node columns up to missing entries), the blocks are >= 70 % filled and
// it streams fewer bytes than `other_bytes` (the storage finalize chose).
bool build_bsr(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes) {
    m.bsr_data.release();
    m.bsr_row0.release();
    m.bsr_soff.release();
    m.bsr_slices = m.bsr_steps = 0;
    m.bsr_seg_slc.clear();
    if (g_spmv_format_policy != 0 || bsr_disabled() || m.no_bsr || m.nnz == 0) return false;
    if (m.nrows % BSR_B || m.ncols % BSR_B || m.nrows < 3 * BSR_C) return false;
    for (int64_t b : m.seg_rows)
        if (b % BSR_B) return false;
    const int64_t N = m.nrows / BSR_B;
    hipStream_t s = m.ctx->stream;
    if (!m.bsr_pin) {  // cheap pre-check on the first node rows: blocked at all?
        const int64_t Ns = std::min<int64_t>(N, 2048), ne = rp[3 * Ns];
        std::vector<int32_t> c(ne);
        if (ne) FAMG_CHECK_HIP(hipMemcpyAsync(c.data(), m.col.get(), ne * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        int64_t blocks = 0;
        for (int64_t I = 0; I < Ns; I++) {
            std::vector<int32_t> u;
            for (int64_t e = rp[3 * I]; e < rp[3 * I + 3]; e++) u.push_back(c[e] / 3);
            std::sort(u.begin(), u.end());
            blocks += std::unique(u.begin(), u.end()) - u.begin();
        }
        if ((double)ne < 0.7 * 9.0 * (double)blocks) return false;
    }
    std::vector<int32_t> col(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    // a renumbered copy (reorder.hip: nodes renumbered, each row in its original
    // order) merges a node's rows by original column: key(c) -- blocks keep their
    // original ascending-column order, stored under the new node column c / 3
    const std::vector<int32_t> &co = m.col_orig;
    auto key = [&](int32_t c) -> int64_t { return co.empty() ? c : co[c]; };
    // node columns per node row: the union of its three rows' (ascending) col / 3
    std::vector<int64_t> nb(N + 1, 0);
    bool sorted = true;
#pragma omp parallel for schedule(static) reduction(&& : sorted)
    for (int64_t I = 0; I < N; I++) {
        int64_t p[3], e[3];
        for (int r = 0; r < 3; r++) { p[r] = rp[3 * I + r]; e[r] = rp[3 * I + r + 1]; }
        int64_t cnt = 0, last = -1;
        for (;;) {
            int64_t best = INT64_MAX;
            for (int r = 0; r < 3; r++)
                if (p[r] < e[r]) best = std::min<int64_t>(best, key(col[p[r]]) / 3);
            if (best == INT64_MAX) break;
            for (int r = 0; r < 3; r++)
                while (p[r] < e[r] && key(col[p[r]]) / 3 == best) p[r]++;
            if (best <= last) sorted = false;
            last = best;
            cnt++;
        }
        nb[I + 1] = cnt;
    }
    if (!sorted) return false;
    for (int64_t I = 0; I < N; I++) nb[I + 1] += nb[I];
    const int64_t nblocks = nb[N];
    if ((double)m.nnz < 0.7 * 9.0 * (double)nblocks) return false;  // too sparse inside the blocks
    // slices of <= 64 node rows that never straddle a row segment
    std::vector<int32_t> row0;
    std::vector<int64_t> seg_slc{0};
    for (size_t g = 0; g + 1 < m.seg_rows.size(); g++) {
        for (int64_t I = m.seg_rows[g] / 3; I < m.seg_rows[g + 1] / 3; I += BSR_C) row0.push_back((int32_t)I);
        seg_slc.push_back((int64_t)row0.size());
    }
    row0.push_back((int32_t)N);
    const int64_t ns = (int64_t)row0.size() - 1;
    std::vector<int32_t> soff(ns + 1, 0);
    for (int64_t k = 0; k < ns; k++) {
        int64_t w = 0;
        for (int64_t I = row0[k]; I < row0[k + 1]; I++) w = std::max<int64_t>(w, nb[I + 1] - nb[I]);
        FAMG_REQUIRE(soff[k] + w < (int64_t(1) << 31), AMG_ERR_UNSUPPORTED, "bsr: too many steps");
        soff[k + 1] = (int32_t)(soff[k] + w);
    }
    const int64_t steps = soff[ns];
    const int64_t bytes = steps * BSR_STEP + 4 * (2 * ns + 2);
    if (bytes >= other_bytes && !m.bsr_pin) return false;
    std::vector<double> val(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), m.val.get(), m.nnz * sizeof(double), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    std::vector<char> data((size_t)steps * BSR_STEP, 0);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t k = 0; k < ns; k++) {
        char *blk = data.data() + (int64_t)soff[k] * BSR_STEP;
        const int64_t w = soff[k + 1] - soff[k];
        for (int64_t I = row0[k]; I < row0[k + 1]; I++) {
            const int lane = (int)(I - row0[k]);
            int64_t p[3], e[3];
            for (int r = 0; r < 3; r++) { p[r] = rp[3 * I + r]; e[r] = rp[3 * I + r + 1]; }
            int64_t t = 0;
            int32_t lastJ = 0;
            for (;; t++) {
                int64_t J = INT64_MAX;
                for (int r = 0; r < 3; r++)
                    if (p[r] < e[r]) J = std::min<int64_t>(J, key(col[p[r]]) / 3);
                if (J == INT64_MAX) break;
                char *st = blk + t * BSR_STEP;
                int32_t Jstore = -1;
                for (int r = 0; r < 3; r++)
                    for (; p[r] < e[r] && key(col[p[r]]) / 3 == J; p[r]++) {
                        Jstore = col[p[r]] / 3;
                        const int kk = 3 * r + col[p[r]] % 3;
                        double *dst = kk < 8 ? reinterpret_cast<double *>(st + (kk / 2) * 1024) + 2 * lane + (kk & 1)
                                             : reinterpret_cast<double *>(st + BSR_K8) + lane;
                        *dst = val[p[r]];
                    }
                reinterpret_cast<int32_t *>(st + BSR_COL)[lane] = Jstore;  // the (new) node column
                lastJ = Jstore;
            }
            for (; t < w; t++)  // padding blocks: zeros at the row's last node column
                reinterpret_cast<int32_t *>(blk + t * BSR_STEP + BSR_COL)[lane] = lastJ;
        }
        for (int lane = (int)(row0[k + 1] - row0[k]); lane < BSR_C; lane++)  // empty lanes
            for (int64_t t = 0; t < w; t++) reinterpret_cast<int32_t *>(blk + t * BSR_STEP + BSR_COL)[lane] = 0;
    }
    m.bsr_data.resize(std::max<size_t>(data.size(), 16));
    m.bsr_row0.resize(ns + 1);
    m.bsr_soff.resize(ns + 1);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.bsr_data.get(), data.data(), data.size(), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.bsr_row0.get(), row0.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.bsr_soff.get(), soff.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.bsr_slices = ns;
    m.bsr_steps = steps;
    m.bsr_maxw = 0;
    for (int64_t k = 0; k < ns; k++) m.bsr_maxw = std::max<int64_t>(m.bsr_maxw, soff[k + 1] - soff[k]);
    m.bsr_seg_slc = seg_slc;
    return true;
}

void spmv_bsr(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg) {
    const int64_t s0 = seg < 0 ? 0 : m.bsr_seg_slc[seg];
    const int64_t s1 = seg < 0 ? m.bsr_slices : m.bsr_seg_slc[seg + 1];
    if (s1 <= s0) return;
    static const int32_t jmask = [] {
        const char *e = getenv("FAMG_BSR_DIAG");
        return (e && e[0] == '1') ? 0 : -1;
    }();
    BsrArgs a{m.bsr_data.get(), m.bsr_row0.get(), m.bsr_soff.get(), (int32_t)s0, (int32_t)(s1 - s0),
              BsrEpi{x, y, epi.b, epi.d, epi.dc, epi.dt, epi.y2}, jmask};
    const dim3 grid((unsigned)ceil_div(s1 - s0, 4)), block(256);
    // T: the template arguments after the mode
#define FAMG_BSR_LAUNCH(K, T)                                                      \
    switch (mode) {                                                                \
    case SPMV_SET: K<SPMV_SET T><<<grid, block, 0, s>>>(a); break;                 \
    case SPMV_ADD: K<SPMV_ADD T><<<grid, block, 0, s>>>(a); break;                 \
    case SPMV_RESID: K<SPMV_RESID T><<<grid, block, 0, s>>>(a); break;             \
    case SPMV_JACOBI: K<SPMV_JACOBI T><<<grid, block, 0, s>>>(a); break;           \
    case SPMV_SETDF: K<SPMV_SETDF T><<<grid, block, 0, s>>>(a); break;             \
    default: fail(AMG_ERR_UNSUPPORTED, "block storage: unsupported SpMV epilogue"); \
    }
#define FAMG_C ,
    const int64_t how = m.bsr_maxw <= BSR_PCOL ? flag(FLAG_BSR_KERNEL) : 0;
    const int64_t lg = flag(FLAG_BSR_LONG);
    // one-wave workgroups below 4096 slices (C5: 1097 -> 1165 V-cycles/s,
    // profiles/r05/ab_bsr_one_wave.txt)
    const bool one = s1 - s0 < BSR_ONE_WAVE_SLICES;  // (everywhere: neutral on C5's A_0)
    const dim3 grid1((unsigned)(s1 - s0)), block1(64);
    if (lg >= 0 && m.bsr_steps >= lg * m.bsr_slices) {
        if (one) {
            const dim3 grid = grid1, block = block1;
            FAMG_BSR_LAUNCH(spmv_bsr3l_kernel, FAMG_C 1)
        } else {
            FAMG_BSR_LAUNCH(spmv_bsr3l_kernel, FAMG_C 4)
        }
    }
    else if (how == 1) FAMG_BSR_LAUNCH(spmv_bsr3p_kernel, FAMG_C 4 FAMG_C false)
    else if (how == 2) FAMG_BSR_LAUNCH(spmv_bsr3p_kernel, FAMG_C 2 FAMG_C true)
    else if (how == 3) FAMG_BSR_LAUNCH(spmv_bsr3p_kernel, FAMG_C 4 FAMG_C true)
    else if (one) {
        const dim3 grid = grid1, block = block1;
        FAMG_BSR_LAUNCH(spmv_bsr3_kernel, FAMG_C 1)
    } else FAMG_BSR_LAUNCH(spmv_bsr3_kernel, FAMG_C 4)
#undef FAMG_BSR_LAUNCH
#undef FAMG_C
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
