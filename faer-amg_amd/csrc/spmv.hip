// spmv.hip -- fp64 CSR SpMV for gfx950 with fused V-cycle epilogues.
//
// Replaces the reference's CPU SpMV (ParSpmmOp, par_spmm.rs:98-133, and faer's
// SparseRowMat LinOp used at multigrid.rs:137-158) and fuses the vector work of
// Multigrid::cycle / smooth (multigrid.rs:341-350, 407-424) into its epilogue.
//
// Design ("CSR-stream", MI355X-first):
//  * The row space is cut on the host into blocks of <= 256 rows holding
//    <= SPMV_CAP nonzeros (GpuCsr::sched).  A 256-thread workgroup streams its
//    block's values and column indices HBM -> LDS with 16-byte, fully coalesced,
//    non-temporal loads (they are read exactly once), then computes rows out of
//    LDS.  x is gathered through L1/L2 (it is re-read by neighbouring rows).
//  * Rows per block decide the lanes per row L (a power of two, L*rows <= 256):
//    short rows (7-pt: 256 rows, L = 1) are summed by one lane sequentially in
//    ascending column order with fma -- bit-identical to the oracle -- while long
//    rows (Galerkin 125-pt, R) spread over L lanes and finish with a shuffle tree.
//    A single row longer than SPMV_CAP gets a whole workgroup.
//  * Workgroups are remapped so that each XCD (blocks b and b+8 share one) walks
//    a contiguous slab of rows: the x window of a slab (3 planes of a 7-pt
//    operator, ~1.5 MB at 256^3) then stays in that XCD's 4 MB L2.
#include "famg.hpp"

namespace famg {

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));

constexpr int SPMV_BS = 256;
constexpr int SPMV_CAP = 2048;

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, idx = b >> 3;
    return x * q + min(x, r) + idx;
}

struct SpmvArgs {
    const int32_t *rowptr;
    const int32_t *col;
    const double *val;
    const int32_t *sched;
    int32_t nblocks;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const int32_t *perm;
};

template <int MODE>
__device__ __forceinline__ void spmv_epilogue(const SpmvArgs &a, int row, double acc) {
    if constexpr (MODE == SPMV_SET) {
        a.y[row] = acc;
    } else if constexpr (MODE == SPMV_ADD) {
        a.y[row] = a.y[row] + acc;
    } else if constexpr (MODE == SPMV_RESID) {
        a.y[row] = a.b[row] - acc;
    } else if constexpr (MODE == SPMV_JACOBI) {
        a.y[row] = a.x[row] + a.d[row] * (a.b[row] - acc);
    } else {  // SPMV_SGS: row is the permuted index
        const int i = a.perm[row];
        a.y[i] = a.x[i] + a.d[row] * (a.b[i] - acc);
    }
}

template <int MODE>
__global__ __launch_bounds__(SPMV_BS) void spmv_stream_kernel(SpmvArgs a) {
    __shared__ __attribute__((aligned(16))) double sval[SPMV_CAP + 2];
    __shared__ __attribute__((aligned(16))) int32_t scol[SPMV_CAP + 4];
    __shared__ double sred[SPMV_BS / 64];

    const int blk = xcd_remap(blockIdx.x, a.nblocks);
    const int r0 = a.sched[blk], r1 = a.sched[blk + 1];
    const int e0 = a.rowptr[r0], e1 = a.rowptr[r1];
    const int tid = threadIdx.x;
    const int nnz = e1 - e0;

    if (nnz > SPMV_CAP) {
        // one long row (r1 == r0 + 1): the whole workgroup reduces it
        double acc = 0.0;
        for (int k = e0 + tid; k < e1; k += SPMV_BS) acc = fma(a.val[k], a.x[a.col[k]], acc);
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if ((tid & 63) == 0) sred[tid >> 6] = acc;
        __syncthreads();
        if (tid == 0) {
            double s = sred[0];
            for (int w = 1; w < SPMV_BS / 64; w++) s += sred[w];
            spmv_epilogue<MODE>(a, r0, s);
        }
        return;
    }

    // ---- stage values and column indices (16-byte coalesced, non-temporal)
    const int bv = e0 & ~1;
    const int nv = (e1 - bv + 1) >> 1;
    const dbl2_t *gv = reinterpret_cast<const dbl2_t *>(a.val + bv);
    dbl2_t *sv2 = reinterpret_cast<dbl2_t *>(sval);
    for (int k = tid; k < nv; k += SPMV_BS) sv2[k] = __builtin_nontemporal_load(gv + k);
    const int bc = e0 & ~3;
    const int nc = (e1 - bc + 3) >> 2;
    const i32x4_t *gc = reinterpret_cast<const i32x4_t *>(a.col + bc);
    i32x4_t *sc4 = reinterpret_cast<i32x4_t *>(scol);
    for (int k = tid; k < nc; k += SPMV_BS) sc4[k] = __builtin_nontemporal_load(gc + k);
    __syncthreads();

    const int nrows = r1 - r0;
    int L = 1;
    while (L < 64 && 2 * L * nrows <= SPMV_BS) L <<= 1;
    const int rl = tid / L;
    const int sub = tid & (L - 1);
    const int vo = e0 - bv, co = e0 - bc;

    double acc = 0.0;
    if (rl < nrows) {
        const int rs = a.rowptr[r0 + rl] - e0;
        const int re = a.rowptr[r0 + rl + 1] - e0;
        for (int k = rs + sub; k < re; k += L) acc = fma(sval[vo + k], a.x[scol[co + k]], acc);
    }
    for (int off = L >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (rl < nrows && sub == 0) spmv_epilogue<MODE>(a, r0 + rl, acc);
}

// ------------------------------------------------------------- SELL-64
//
// Short regular rows (7-pt fine level, P): one lane per row, one wavefront per
// 64-row slice.  The slice is stored column-major, so entry k of the 64 rows is
// one 512-B (values) / 256-B (columns) contiguous access; there is no LDS, no
// barrier and no row-pointer traffic (one offset per 64 rows).  All loads of a
// chunk of up to 8 entries are issued before the dependent x gathers, and the
// epilogue operands are fetched first, so each lane keeps ~20 loads in flight.
// The row sum is still sequential in ascending column order (padding adds
// 0 * x[c_last]), i.e. bit-identical to the oracle.

int g_spmv_format_policy = 0;
constexpr int SELL_C = 64;
constexpr int SELL_MAX_W = 48;

struct SellArgs {
    const int32_t *off;
    const int32_t *col;
    const double *val;
    int32_t nslices;
    int32_t nrows;
    const double *x;
    double *y;
    const double *b;
    const double *d;
};

template <int U>
__device__ __forceinline__ void sell_chunk(const double *__restrict__ v, const int32_t *__restrict__ c,
                                           const double *__restrict__ x, double &acc) {
    double vv[U];
    int32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        vv[u] = __builtin_nontemporal_load(v + u * SELL_C);
        cc[u] = __builtin_nontemporal_load(c + u * SELL_C);
    }
    double xx[U];
#pragma unroll
    for (int u = 0; u < U; u++) xx[u] = x[cc[u]];
#pragma unroll
    for (int u = 0; u < U; u++) acc = fma(vv[u], xx[u], acc);
}

template <int MODE>
__global__ __launch_bounds__(256) void spmv_sell_kernel(SellArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int slice = blk * 4 + (threadIdx.x >> 6);
    if (slice >= a.nslices) return;
    const int lane = threadIdx.x & 63;
    const int row = slice * SELL_C + lane;
    const bool live = row < a.nrows;
    double xr = 0.0, br = 0.0, dr = 0.0, yr = 0.0;
    if (live) {
        if constexpr (MODE == SPMV_JACOBI) { xr = a.x[row]; br = a.b[row]; dr = a.d[row]; }
        if constexpr (MODE == SPMV_RESID) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
    }
    const int o0 = a.off[slice];
    const int w = (a.off[slice + 1] - o0) >> 6;
    const double *v = a.val + o0 + lane;
    const int32_t *c = a.col + o0 + lane;
    double acc = 0.0;
    int k = 0;
    for (; k + 8 <= w; k += 8) sell_chunk<8>(v + k * SELL_C, c + k * SELL_C, a.x, acc);
    v += k * SELL_C;
    c += k * SELL_C;
    switch (w - k) {
    case 1: sell_chunk<1>(v, c, a.x, acc); break;
    case 2: sell_chunk<2>(v, c, a.x, acc); break;
    case 3: sell_chunk<3>(v, c, a.x, acc); break;
    case 4: sell_chunk<4>(v, c, a.x, acc); break;
    case 5: sell_chunk<5>(v, c, a.x, acc); break;
    case 6: sell_chunk<6>(v, c, a.x, acc); break;
    case 7: sell_chunk<7>(v, c, a.x, acc); break;
    default: break;
    }
    if (!live) return;
    if constexpr (MODE == SPMV_SET) a.y[row] = acc;
    else if constexpr (MODE == SPMV_ADD) a.y[row] = yr + acc;
    else if constexpr (MODE == SPMV_RESID) a.y[row] = br - acc;
    else if constexpr (MODE == SPMV_JACOBI) a.y[row] = xr + dr * (br - acc);
}

__global__ void k_sell_fill(const int64_t *rp, const int32_t *col, const double *val, int64_t n,
                            const int32_t *off, int64_t nslices, int32_t *scol, double *sval) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= nslices * SELL_C) return;
    const int64_t s = r / SELL_C, lane = r % SELL_C;
    const int64_t len = r < n ? rp[r + 1] - rp[r] : 0;
    const int64_t base = r < n ? rp[r] : 0;
    const int w = (off[s + 1] - off[s]) / SELL_C;
    const int32_t cpad = len > 0 ? col[base + len - 1] : 0;
    for (int k = 0; k < w; k++) {
        const int64_t o = off[s] + (int64_t)k * SELL_C + lane;
        if (k < len) { scol[o] = col[base + k]; sval[o] = val[base + k]; }
        else { scol[o] = cpad; sval[o] = 0.0; }
    }
}

void build_sell(GpuCsr &m, const std::vector<int64_t> &rp) {
    m.sell_off.release();
    m.sell_col.release();
    m.sell_val.release();
    m.nslices = m.sell_padded = 0;
    if (g_spmv_format_policy == 1 || m.nrows == 0 || m.nnz == 0) return;
    const int64_t ns = ceil_div(m.nrows, SELL_C);
    std::vector<int32_t> off(ns + 1, 0);
    int64_t padded = 0, maxw = 0;
    for (int64_t s = 0; s < ns; s++) {
        int64_t w = 0;
        const int64_t r1 = std::min<int64_t>(m.nrows, (s + 1) * SELL_C);
        for (int64_t r = s * SELL_C; r < r1; r++) w = std::max<int64_t>(w, rp[r + 1] - rp[r]);
        maxw = std::max(maxw, w);
        padded += w * SELL_C;
        if (padded >= (int64_t(1) << 31)) return;
        off[s + 1] = static_cast<int32_t>(padded);
    }
    const bool ok = g_spmv_format_policy == 2 ? maxw <= 256
                                              : (maxw <= SELL_MAX_W && padded * 100 <= m.nnz * 112);
    if (!ok) return;
    hipStream_t s = m.ctx->stream;
    m.sell_off.resize(ns + 1);
    m.sell_col.resize(padded);
    m.sell_val.resize(padded);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_off.get(), off.data(), (ns + 1) * sizeof(int32_t),
                                  hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_sell_fill, dim3((unsigned)ceil_div(ns * SELL_C, 256)), dim3(256), 0, s,
                       m.rp64.get(), m.col.get(), m.val.get(), m.nrows, m.sell_off.get(), ns,
                       m.sell_col.get(), m.sell_val.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.nslices = ns;
    m.sell_padded = padded;
}

static void spmv_sell(const GpuCsr &m, const double *x, double *y, SpmvMode mode,
                      const SpmvEpi &epi, hipStream_t s) {
    SellArgs a;
    a.off = m.sell_off.get();
    a.col = m.sell_col.get();
    a.val = m.sell_val.get();
    a.nslices = static_cast<int32_t>(m.nslices);
    a.nrows = static_cast<int32_t>(m.nrows);
    a.x = x;
    a.y = y;
    a.b = epi.b;
    a.d = epi.d;
    dim3 grid(static_cast<unsigned>(ceil_div(m.nslices, 4))), block(256);
    switch (mode) {
    case SPMV_SET: hipLaunchKernelGGL(spmv_sell_kernel<SPMV_SET>, grid, block, 0, s, a); break;
    case SPMV_ADD: hipLaunchKernelGGL(spmv_sell_kernel<SPMV_ADD>, grid, block, 0, s, a); break;
    case SPMV_RESID: hipLaunchKernelGGL(spmv_sell_kernel<SPMV_RESID>, grid, block, 0, s, a); break;
    case SPMV_JACOBI: hipLaunchKernelGGL(spmv_sell_kernel<SPMV_JACOBI>, grid, block, 0, s, a); break;
    default: fail(AMG_ERR_INVALID, "SELL SpMV: unsupported mode");
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

void spmv(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
          hipStream_t s, int64_t blk_begin, int64_t blk_end, const int32_t *sched_override) {
    FAMG_REQUIRE(m.spmv_ready(), AMG_ERR_UNSUPPORTED,
                 "SpMV needs nnz < 2^31 (32-bit row pointers)");
    if (m.has_sell() && mode != SPMV_SGS && blk_begin == 0 && blk_end < 0 && !sched_override) {
        spmv_sell(m, x, y, mode, epi, s);
        return;
    }
    if (blk_end < 0) blk_end = m.nblocks;
    const int64_t nb = blk_end - blk_begin;
    if (nb <= 0) return;
    SpmvArgs a;
    a.rowptr = m.rp32.get();
    a.col = m.col.get();
    a.val = m.val.get();
    a.sched = (sched_override ? sched_override : m.sched.get()) + blk_begin;
    a.nblocks = static_cast<int32_t>(nb);
    a.x = x;
    a.y = y;
    a.b = epi.b;
    a.d = epi.d;
    a.perm = epi.perm;
    dim3 grid(static_cast<unsigned>(nb)), block(SPMV_BS);
    switch (mode) {
    case SPMV_SET: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_SET>, grid, block, 0, s, a); break;
    case SPMV_ADD: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_ADD>, grid, block, 0, s, a); break;
    case SPMV_RESID: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_RESID>, grid, block, 0, s, a); break;
    case SPMV_JACOBI: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_JACOBI>, grid, block, 0, s, a); break;
    case SPMV_SGS: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_SGS>, grid, block, 0, s, a); break;
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

// Host-side schedule: greedy blocks of <= SPMV_BS rows and <= SPMV_CAP nonzeros;
// a row longer than SPMV_CAP is a block of its own.  Blocks never cross the
// given segment boundaries (SGS colors).
void build_schedule(const std::vector<int64_t> &rp, const std::vector<int64_t> &seg_bounds,
                    std::vector<int32_t> &sched, std::vector<int64_t> &seg_blocks) {
    sched.clear();
    seg_blocks.clear();
    sched.push_back(static_cast<int32_t>(seg_bounds.empty() ? 0 : seg_bounds[0]));
    seg_blocks.push_back(0);
    for (size_t s = 0; s + 1 < seg_bounds.size(); s++) {
        int64_t r0 = seg_bounds[s];
        const int64_t end = seg_bounds[s + 1];
        while (r0 < end) {
            int64_t r1;
            if (rp[r0 + 1] - rp[r0] > SPMV_CAP) {
                r1 = r0 + 1;
            } else {
                r1 = r0;
                while (r1 < end && r1 - r0 < SPMV_BS && rp[r1 + 1] - rp[r0] <= SPMV_CAP) r1++;
            }
            sched.push_back(static_cast<int32_t>(r1));
            r0 = r1;
        }
        seg_blocks.push_back(static_cast<int64_t>(sched.size()) - 1);
    }
}

}  // namespace famg
