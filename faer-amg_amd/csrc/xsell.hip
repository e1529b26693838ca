// xsell.hip -- x-staged SELL for gather-heavy general operators.
//
// A general sparse matrix whose rows are not stored in a locality-preserving
// order (the roofline.general operator: random coefficients, rows shuffled
// within windows of 4096) gathers every x operand from a different cache line:
// on gfx950 each 8-B gather pulls a 128-B line from L2 into L1, and with three
// 32-KB x windows per row group against a 32-KB L1 those fills, not HBM, bound
// the SpMV (SELL with u16/i32 columns: 0.47 ms for 1.25 GB of matrix stream).
//
// Here the x footprint of each group of 64 slices (4096 rows) is copied once
// into LDS and the row sums read it there.  Group g stages up to XS_MAXCH
// chunks of 64 consecutive x entries (512 B; 160 KB, the whole LDS of a CU):
// the chunks its entries reference, the most referenced first.  A slice whose
// entries all fall in staged chunks stores a 16-bit LDS index per entry
// (slot * 64 + column % 64); a slice with any entry outside them keeps 32-bit
// global columns (escape slices, gathered through the caches).  Values stay
// fp64, one step per 512-B row per slice (step t of lane l at t * 64 + l), the
// index block after the values.
//
// One 1024-thread workgroup per group: the 16 waves stage the chunks (16-B
// loads), meet at one barrier, then each wave walks slices w, w + 16, w + 32,
// w + 48 of the group, 8 steps at a time with all value/index loads of a step
// group issued before the LDS (or global) gathers.  A row's sum runs over its
// stored entries in order with fma -- the oracle's order, bitwise.  Padding
// steps add fma(0.0, x, acc) with an in-range staged x.
//
// Every mode but SGS (whose color-permuted copies never get this storage): the
// folded zero-guess residual stages d*x (the product vec_mul would store), the
// folded correction adds d*b in its epilogue.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "famg.hpp"

namespace famg {

typedef double xs_dbl2_t __attribute__((ext_vector_type(2)));

constexpr int XS_SLICES = 64;                // slices per group (4096 rows)
constexpr int XS_ROWS = XS_SLICES * 64;
constexpr int XS_CH = 64;                    // x entries per chunk
constexpr int XS_MAXCH = 320;                // chunks per group (160 KB: all of the LDS)
constexpr int XS_BS = 1024;                  // threads per workgroup
constexpr int XS_MAX_W = 64;                 // widest slice stored

struct XsArgs {
    const char *data;       // per slice: values (w x 64 fp64) then indices (w x 64 u16 / i32)
    const uint32_t *desc;   // per slice: byte offset / 128 | mode << 30 (1: LDS u16, 2: global i32)
    const int32_t *soff;    // per slice: first step (+1 sentinel); w = soff[s+1] - soff[s]
    const int32_t *coff;    // per group: first chunk (+1 sentinel)
    const int32_t *chunks;  // staged chunk ids, per group ascending
    int32_t nrows, ncols, ngroups;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
};

// all loads of U steps issued before the gathers, then U fmas in step order
template <int CM, int MODE, int U>
__device__ __forceinline__ void xs_steps(const char *__restrict__ blk, int w, int t0, int lane,
                                         const double *__restrict__ sx, const XsArgs &a, double &acc) {
    double v[U], xv[U];
    int32_t ix[U];
    const double *vp = reinterpret_cast<const double *>(blk) + (int64_t)t0 * 64 + lane;
#pragma unroll
    for (int u = 0; u < U; u++) {
        v[u] = __builtin_nontemporal_load(vp + u * 64);
        if constexpr (CM == 1)
            ix[u] = __builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(blk + (int64_t)w * 512) +
                                               (int64_t)(t0 + u) * 64 + lane);
        else
            ix[u] = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(blk + (int64_t)w * 512) +
                                               (int64_t)(t0 + u) * 64 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if constexpr (CM == 1) xv[u] = sx[ix[u]];
        else if constexpr (MODE == SPMV_RESID0) xv[u] = a.d[ix[u]] * a.x[ix[u]];
        else xv[u] = a.x[ix[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc = fma(v[u], xv[u], acc);
}

template <int CM, int MODE>
__device__ __forceinline__ double xs_walk(const char *blk, int w, int lane, const double *sx, const XsArgs &a) {
    double acc = 0.0;
    int t = 0;
    for (; t + 8 <= w; t += 8) xs_steps<CM, MODE, 8>(blk, w, t, lane, sx, a, acc);
    switch (w - t) {
    case 1: xs_steps<CM, MODE, 1>(blk, w, t, lane, sx, a, acc); break;
    case 2: xs_steps<CM, MODE, 2>(blk, w, t, lane, sx, a, acc); break;
    case 3: xs_steps<CM, MODE, 3>(blk, w, t, lane, sx, a, acc); break;
    case 4: xs_steps<CM, MODE, 4>(blk, w, t, lane, sx, a, acc); break;
    case 5: xs_steps<CM, MODE, 5>(blk, w, t, lane, sx, a, acc); break;
    case 6: xs_steps<CM, MODE, 6>(blk, w, t, lane, sx, a, acc); break;
    case 7: xs_steps<CM, MODE, 7>(blk, w, t, lane, sx, a, acc); break;
    default: break;
    }
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(XS_BS) void spmv_xs_kernel(XsArgs a) {
    __shared__ double sx[XS_MAXCH * XS_CH];
    const int g = xcd_remap(blockIdx.x, gridDim.x);
    const int c0 = a.coff[g], nch = a.coff[g + 1] - c0;
    for (int i = threadIdx.x; i < nch * (XS_CH / 2); i += XS_BS) {
        const int64_t e = (int64_t)a.chunks[c0 + i / (XS_CH / 2)] * XS_CH + 2 * (i % (XS_CH / 2));
        xs_dbl2_t v = {0.0, 0.0};
        if (e + 1 < a.ncols) v = *reinterpret_cast<const xs_dbl2_t *>(a.x + e);
        else if (e < a.ncols) v.x = a.x[e];
        if constexpr (MODE == SPMV_RESID0) {  // the x operand is the zero-guess iterate d*x (vec_mul's product)
            xs_dbl2_t dv = {0.0, 0.0};
            if (e + 1 < a.ncols) dv = *reinterpret_cast<const xs_dbl2_t *>(a.d + e);
            else if (e < a.ncols) dv.x = a.d[e];
            v = dv * v;
        }
        *reinterpret_cast<xs_dbl2_t *>(sx + 2 * i) = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int s_end = min((g + 1) * XS_SLICES, (a.nrows + 63) / 64);
    for (int s = g * XS_SLICES + wave; s < s_end; s += XS_BS / 64) {
        const int row = s * 64 + lane;
        const bool live = row < a.nrows;
        double xr = 0.0, br = 0.0, dr = 0.0, yr = 0.0;  // epilogue operands first
        if (live) {
            if constexpr (MODE == SPMV_JACOBI) {
                xr = a.x[row];
                dr = a.dc ? a.dt[a.dc[row]] : a.d[row];
            }
            if constexpr (MODE == SPMV_JACOBI || MODE == SPMV_RESID || MODE == SPMV_RESID0) br = a.b[row];
            if constexpr (MODE == SPMV_ADD) yr = a.y[row];
            if constexpr (MODE == SPMV_ADD0) yr = (a.dc ? a.dt[a.dc[row]] : a.d[row]) * a.b[row];
        }
        const int w = a.soff[s + 1] - a.soff[s];
        const uint32_t d = a.desc[s];
        const char *blk = a.data + (int64_t)(d & 0x3fffffffu) * 128;
        // escape slices gather x (RESID0: d*x) through the caches
        const double acc = (d >> 30) == 1 ? xs_walk<1, MODE>(blk, w, lane, sx, a) : xs_walk<2, MODE>(blk, w, lane, sx, a);
        if (live) {
            if constexpr (MODE == SPMV_SET) a.y[row] = acc;
            else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[row] = yr + acc;
            else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[row] = br - acc;
            else a.y[row] = xr + dr * (br - acc);  // JACOBI
        }
    }
}

// ---------------------------------------------------------------- multi-column
// Y = A X for k columns (f2, adaptivity.rs:168-244): one workgroup per group
// walks its slices once per column with that column's chunks staged in LDS --
// exactly the single-vector kernel's sums (bitwise per column), the group's
// matrix read from HBM once and re-read from L2 / MALL for the other columns
// (one x window fits the LDS, eight do not).
__global__ __launch_bounds__(XS_BS) void spmm_xs_group_kernel(XsArgs a, int kb, int64_t ldx, int64_t ldy) {
    __shared__ double sx[XS_MAXCH * XS_CH];
    const int g = xcd_remap(blockIdx.x, gridDim.x);
    const int c0 = a.coff[g], nch = a.coff[g + 1] - c0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int s_end = min((g + 1) * XS_SLICES, (a.nrows + 63) / 64);
    const double *x0 = a.x;
    double *y0 = a.y;
    for (int c = 0; c < kb; c++) {
        a.x = x0 + c * ldx;
        a.y = y0 + c * ldy;
        if (c) __syncthreads();  // the previous column's walk is done with sx
        for (int i = threadIdx.x; i < nch * (XS_CH / 2); i += XS_BS) {
            const int64_t e = (int64_t)a.chunks[c0 + i / (XS_CH / 2)] * XS_CH + 2 * (i % (XS_CH / 2));
            xs_dbl2_t v = {0.0, 0.0};
            if (e + 1 < a.ncols) v = *reinterpret_cast<const xs_dbl2_t *>(a.x + e);
            else if (e < a.ncols) v.x = a.x[e];
            *reinterpret_cast<xs_dbl2_t *>(sx + 2 * i) = v;
        }
        __syncthreads();
        for (int s = g * XS_SLICES + wave; s < s_end; s += XS_BS / 64) {
            const int row = s * 64 + lane;
            const int w = a.soff[s + 1] - a.soff[s];
            const uint32_t d = a.desc[s];
            const char *blk = a.data + (int64_t)(d & 0x3fffffffu) * 128;
            const double acc = (d >> 30) == 1 ? xs_walk<1, SPMV_SET>(blk, w, lane, sx, a)
                                              : xs_walk<2, SPMV_SET>(blk, w, lane, sx, a);
            if (row < a.nrows) a.y[row] = acc;
        }
    }
}

bool spmm_xs(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k, hipStream_t s) {
    if (m.kernel != SPMV_KERNEL_XS || !m.has_xs()) return false;
    if (m.nrows == 0 || k == 0) return true;
    XsArgs a{};
    a.data = m.xs_data.get();
    a.desc = m.xs_desc.get();
    a.soff = m.xs_soff.get();
    a.coff = m.xs_coff.get();
    a.chunks = m.xs_chunks.get();
    a.nrows = (int32_t)m.nrows;
    a.ncols = (int32_t)m.ncols;
    a.ngroups = (int32_t)m.xs_groups;
    for (int64_t c0 = 0; c0 < k; c0 += 8) {
        a.x = x + c0 * ldx;
        a.y = y + c0 * ldy;
        spmm_xs_group_kernel<<<dim3((unsigned)m.xs_groups), dim3(XS_BS), 0, s>>>(a, (int)std::min<int64_t>(8, k - c0),
                                                                               ldx, ldy);
        FAMG_CHECK_HIP(hipGetLastError());
    }
    return true;
}

// ---------------------------------------------------------------- pipelined form
// The kernel above pays two dependent memory round trips per staging trip (the
// chunk id, then its x entries: ten trips of a 1024-thread workgroup for 320
// chunks) and one round trip per slice walk with nothing else in flight.  Here
// (default; FLAG_XS_PIPE = 0 selects the kernel above):
//  * every wave issues the value/index loads of its first 8-step batch and its
//    first slice's epilogue operands before the staging starts, so the matrix
//    stream runs under the staging;
//  * the staging loads all its chunk ids at once, then all its x pairs, then
//    writes LDS (two round trips per workgroup instead of twenty);
//  * the walk is software pipelined over a wave's batches (8 steps of one slice):
//    batch k + 1's loads are issued before batch k's LDS gathers and fmas.  A
//    batch past the slice's width loads its last step again (clamped, never
//    summed), the batch after the wave's last one reloads that one: no branch
//    around a load, so the compiler counts the loads in flight exactly.
// Per row the same stored entries are summed in the same order: bitwise the
// kernel above.
constexpr int XS_B = 8;                      // steps per batch
constexpr int XS_STAGE = (XS_MAXCH * XS_CH / 2 + XS_BS - 1) / XS_BS;  // 16-B staging loads per thread

template <int NB = XS_B>
struct XsBatch {
    double v[NB];
    int32_t ix[NB];
};

// operands the epilogue of one row needs (loaded with the slice's first batch)
struct XsEpi {
    double x, b, d, y;
};

// a batch's loads: steps t0..t0+7 clamped to the slice's last step (no branch
// around a load: on a control-flow join the compiler's wait counting turns
// conservative).  Escape slices are read the same way (their 32-bit column
// block read as 16-bit halves: in bounds, never summed -- see below).
template <int NB>
__device__ __forceinline__ void xs_issue(XsBatch<NB> &B, const char *blk, int w, int t0, int lane) {
    const double *vp = reinterpret_cast<const double *>(blk) + lane;
    const uint16_t *ip = reinterpret_cast<const uint16_t *>(blk + (int64_t)w * 512) + lane;
    const int tl = w - 1;  // every slice has >= 1 step
#pragma unroll
    for (int u = 0; u < NB; u++) B.v[u] = __builtin_nontemporal_load(vp + (int64_t)min(t0 + u, tl) * 64);
#pragma unroll
    for (int u = 0; u < NB; u++) B.ix[u] = __builtin_nontemporal_load(ip + (int64_t)min(t0 + u, tl) * 64);
}

template <int MODE>
__device__ __forceinline__ XsEpi xs_epi_load(const XsArgs &a, int row) {
    XsEpi e{0.0, 0.0, 0.0, 0.0};
    const int r = min(row, a.nrows - 1);  // padding lanes: any row, never stored
    if constexpr (MODE == SPMV_JACOBI) {
        e.x = a.x[r];
        e.d = a.dc ? a.dt[a.dc[r]] : a.d[r];
    }
    if constexpr (MODE == SPMV_JACOBI || MODE == SPMV_RESID || MODE == SPMV_RESID0) e.b = a.b[r];
    if constexpr (MODE == SPMV_ADD) e.y = a.y[r];
    if constexpr (MODE == SPMV_ADD0) e.y = (a.dc ? a.dt[a.dc[r]] : a.d[r]) * a.b[r];
    return e;
}

// LDS gathers (indices clamped into the window: an escape slice's are not LDS
// indices) and the fmas of the batch's first cnt steps
template <int NB>
__device__ __forceinline__ double xs_consume(const XsBatch<NB> &B, int cnt, const double *sx, double acc) {
    double xv[NB];
#pragma unroll
    for (int u = 0; u < NB; u++) xv[u] = sx[min(B.ix[u], XS_MAXCH * XS_CH - 1)];
#pragma unroll
    for (int u = 0; u < NB; u++)
        if (u < cnt) acc = fma(B.v[u], xv[u], acc);
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(XS_BS) void spmv_xs_pipe_kernel(XsArgs a) {
    __shared__ double sx[XS_MAXCH * XS_CH];
    const int g = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s_end = min((g + 1) * XS_SLICES, (a.nrows + 63) / 64);
    const int s_last = s_end - 1;

    // the wave's first batch and epilogue operands, in flight during the staging
    int s = g * XS_SLICES + wave;
    int sc = min(s, s_last);
    int w = a.soff[sc + 1] - a.soff[sc];
    uint32_t dsc = a.desc[sc];
    XsBatch<> cur;
    xs_issue(cur, a.data + (int64_t)(dsc & 0x3fffffffu) * 128, w, 0, lane);
    XsEpi epi = xs_epi_load<MODE>(a, sc * 64 + lane);

    // staging: all chunk ids, then all x pairs, then the LDS writes
    {
        const int c0 = a.coff[g], nch = a.coff[g + 1] - c0, tot = nch * (XS_CH / 2);
        int32_t ch[XS_STAGE];
#pragma unroll
        for (int k = 0; k < XS_STAGE; k++) {
            const int i = min((int)threadIdx.x + k * XS_BS, tot - 1);
            ch[k] = a.chunks[c0 + i / (XS_CH / 2)];
        }
        xs_dbl2_t v[XS_STAGE];
        const int64_t nc = a.ncols;
#pragma unroll
        for (int k = 0; k < XS_STAGE; k++) {
            const int i = min((int)threadIdx.x + k * XS_BS, tot - 1);
            const int64_t e = (int64_t)ch[k] * XS_CH + 2 * (i % (XS_CH / 2));  // even
            const int64_t ea = min(e, nc - 2);                                   // ncols >= 2: a pair in range
            xs_dbl2_t xv = *reinterpret_cast<const xs_dbl2_t *>(a.x + ea);
            if constexpr (MODE == SPMV_RESID0) xv = *reinterpret_cast<const xs_dbl2_t *>(a.d + ea) * xv;
            // e = nc - 1 (odd nc): the pair loaded is (nc - 2, nc - 1); e >= nc: zeros
            const double lo = e == ea ? xv.x : (e == nc - 1 ? xv.y : 0.0);
            const double hi = e == ea ? xv.y : 0.0;
            v[k] = xs_dbl2_t{lo, hi};
        }
#pragma unroll
        for (int k = 0; k < XS_STAGE; k++) {
            const int i = (int)threadIdx.x + k * XS_BS;
            if (i < tot) *reinterpret_cast<xs_dbl2_t *>(sx + 2 * i) = v[k];
        }
    }
    __syncthreads();

    double acc = 0.0;
    int t0 = 0;
    bool done = s >= s_end;
    // one pipeline step: consume cur, with nxt's loads in flight (two buffers
    // alternate roles, so no register copy waits for the loads)
    // a finished row's y is stored at the start of the next step, before that
    // step's loads: on gfx950 stores count in vmcnt, so a store issued after the
    // loads would make the next register reuse wait for all of them
    int prow = -1;
    double pval = 0.0;
    auto step = [&](const XsBatch<> &cur, XsBatch<> &nxt) {
        if (prow >= 0 && prow < a.nrows) a.y[prow] = pval;
        prow = -1;
        const bool last = t0 + XS_B >= w;
        const int sn = last ? s + XS_BS / 64 : s, tn = last ? 0 : t0 + XS_B;
        // the next batch (the wave's last batch again past its end)
        const bool more = sn < s_end;
        const int snc = min(sn, s_last);
        const int wn = more ? a.soff[snc + 1] - a.soff[snc] : w;
        const uint32_t dn = more ? a.desc[snc] : dsc;
        xs_issue(nxt, a.data + (int64_t)(dn & 0x3fffffffu) * 128, wn, more ? tn : t0, lane);
        const XsEpi en = xs_epi_load<MODE>(a, snc * 64 + lane);
        acc = xs_consume(cur, min(XS_B, w - t0), sx, acc);
        if (last) {
            prow = (dsc >> 30) == 1 ? s * 64 + lane : -1;  // escape slices: below
            if constexpr (MODE == SPMV_SET) pval = acc;
            else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) pval = epi.y + acc;
            else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) pval = epi.b - acc;
            else pval = epi.x + epi.d * (epi.b - acc);  // JACOBI
            acc = 0.0;
            epi = en;
        }
        s = sn;
        t0 = tn;
        w = wn;
        dsc = dn;
        done = !more;
    };
    XsBatch<> alt;
    while (!done) {
        step(cur, alt);
        if (done) break;
        step(alt, cur);
    }
    if (prow >= 0 && prow < a.nrows) a.y[prow] = pval;
    // escape slices (32-bit global columns, at most 1/16 of the slices) gather x
    // through the caches, one slice at a time as in the kernel above
    for (int e = g * XS_SLICES + wave; e < s_end; e += XS_BS / 64) {
        const uint32_t d = a.desc[e];
        if ((d >> 30) == 1) continue;
        const int row = e * 64 + lane;
        const XsEpi ep = xs_epi_load<MODE>(a, row);
        const double acc2 = xs_walk<2, MODE>(a.data + (int64_t)(d & 0x3fffffffu) * 128, a.soff[e + 1] - a.soff[e], lane, sx, a);
        if (row < a.nrows) {
            if constexpr (MODE == SPMV_SET) a.y[row] = acc2;
            else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[row] = ep.y + acc2;
            else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[row] = ep.b - acc2;
            else a.y[row] = ep.x + ep.d * (ep.b - acc2);  // JACOBI
        }
    }
}

// ---------------------------------------------------------------- burst form
// One round trip per group for everything the group reads from HBM (flag
// FLAG_XS_PIPE = 2, the default): every wave first loads the chunk ids of its
// staging share, then issues the first NB-step batch of all four of its slices
// (values + LDS indices: 4 x 3 NB VGPRs) and its epilogue operands, and stages
// its chunk pairs with LDS-DMA (global_load_lds_dwordx4: one wave instruction
// copies two 512-B chunks straight into LDS, no registers), so the group's
// 290 KB of matrix and 160 KB of x window are in flight at once; one barrier,
// then the four slices are summed from registers and LDS.  Slices wider than NB
// steps load their further batches one at a time.  The folded zero-guess
// residual (RESID0) stages d*x, a product, through registers instead.
// Bitwise the kernels above: the same stored entries per row, in order.
constexpr int XS_NS = XS_SLICES / (XS_BS / 64);    // slices per wave (4)
constexpr int XS_PPW = XS_MAXCH / 2 / (XS_BS / 64);  // LDS-DMA chunk pairs per wave (10)

template <int MODE, int NB>
__global__ __launch_bounds__(XS_BS) void spmv_xs_burst_kernel(XsArgs a) {
    __shared__ double sx[XS_MAXCH * XS_CH];
    const int g = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s0 = g * XS_SLICES + wave;
    const int s_end = min((g + 1) * XS_SLICES, (a.nrows + 63) / 64);
    const int s_last = s_end - 1;
    const int c0 = a.coff[g], nch = a.coff[g + 1] - c0;
    const int64_t nc = a.ncols;

    XsBatch<NB> B[XS_NS];
    int W[XS_NS];
#pragma unroll
    for (int j = 0; j < XS_NS; j++) {
        const int sc = min(s0 + 16 * j, s_last);
        W[j] = a.soff[sc + 1] - a.soff[sc];
        xs_issue(B[j], a.data + (int64_t)(a.desc[sc] & 0x3fffffffu) * 128, W[j], 0, lane);
    }
    if constexpr (MODE != SPMV_RESID0) {
        // the chunk ids of the wave's pairs by scalar loads, all before the first
        // LDS-DMA (a scalar load may not follow a write the compiler cannot rule
        // out); counted on lgkmcnt, so the matrix loads in flight are not waited for
        int32_t clo[XS_PPW], chi[XS_PPW];
#pragma unroll
        for (int j = 0; j < XS_PPW; j++) {
            const int p = min(wave + 16 * j, (nch - 1) / 2);
            clo[j] = a.chunks[c0 + 2 * p];
            chi[j] = a.chunks[c0 + min(2 * p + 1, nch - 1)];
        }
#pragma unroll
        for (int j = 0; j < XS_PPW; j++) {
            const int p = wave + 16 * j;
            if (2 * p < nch) {  // wave-uniform: the pair's first chunk exists
                const int slot = 2 * p + (lane >> 5);
                const int64_t e = (int64_t)(lane >> 5 ? chi[j] : clo[j]) * XS_CH + 2 * (lane & 31);
                if (slot < nch && e + 1 < nc)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(a.x + e),
                                                     (__attribute__((address_space(3))) void *)(sx + 2 * p * XS_CH), 16, 0, 0);
                else if (slot < nch && e < nc)
                    sx[slot * XS_CH + 2 * (lane & 31)] = a.x[e];  // odd ncols: the last entry alone
            }
        }
    } else {
        const int tot = nch * (XS_CH / 2);
        for (int i = threadIdx.x; i < tot; i += XS_BS) {
            const int64_t e = (int64_t)a.chunks[c0 + i / (XS_CH / 2)] * XS_CH + 2 * (i % (XS_CH / 2));
            xs_dbl2_t v = {0.0, 0.0};
            if (e + 1 < nc) v = *reinterpret_cast<const xs_dbl2_t *>(a.d + e) * *reinterpret_cast<const xs_dbl2_t *>(a.x + e);
            else if (e < nc) v.x = a.d[e] * a.x[e];
            *reinterpret_cast<xs_dbl2_t *>(sx + 2 * i) = v;
        }
    }
    // epilogue operands: with the burst where registers allow; else (JACOBI's
    // three, or 8-step batches) each slice's right after its batch is summed
    constexpr bool epi_late = MODE == SPMV_JACOBI || (NB > 7 && MODE != SPMV_SET);
    XsEpi E[XS_NS];
    if constexpr (!epi_late) {
#pragma unroll
        for (int j = 0; j < XS_NS; j++) E[j] = xs_epi_load<MODE>(a, min(s0 + 16 * j, s_last) * 64 + lane);
    }
    __syncthreads();
    double acc[XS_NS];
#pragma unroll
    for (int j = 0; j < XS_NS; j++) {
        const int s = min(s0 + 16 * j, s_last);
        const uint32_t dsc = a.desc[s];
        const char *blk = a.data + (int64_t)(dsc & 0x3fffffffu) * 128;
        acc[j] = xs_consume(B[j], min(NB, W[j]), sx, 0.0);
        if constexpr (epi_late) E[j] = xs_epi_load<MODE>(a, s * 64 + lane);
        for (int t0 = NB; t0 < W[j]; t0 += NB) {
            XsBatch<NB> X;
            xs_issue(X, blk, W[j], t0, lane);
            acc[j] = xs_consume(X, min(NB, W[j] - t0), sx, acc[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < XS_NS; j++) {
        const int s = s0 + 16 * j;
        if (s >= s_end) break;
        if ((a.desc[s] >> 30) != 1) continue;  // escape slice: below
        const int row = s * 64 + lane;
        if (row < a.nrows) {
            if constexpr (MODE == SPMV_SET) a.y[row] = acc[j];
            else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[row] = E[j].y + acc[j];
            else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[row] = E[j].b - acc[j];
            else a.y[row] = E[j].x + E[j].d * (E[j].b - acc[j]);  // JACOBI
        }
    }
    for (int e = s0; e < s_end; e += XS_BS / 64) {
        const uint32_t d = a.desc[e];
        if ((d >> 30) == 1) continue;
        const int row = e * 64 + lane;
        const XsEpi ep = xs_epi_load<MODE>(a, row);
        const double acc2 = xs_walk<2, MODE>(a.data + (int64_t)(d & 0x3fffffffu) * 128, a.soff[e + 1] - a.soff[e], lane, sx, a);
        if (row < a.nrows) {
            if constexpr (MODE == SPMV_SET) a.y[row] = acc2;
            else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[row] = ep.y + acc2;
            else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[row] = ep.b - acc2;
            else a.y[row] = ep.x + ep.d * (ep.b - acc2);  // JACOBI
        }
    }
}

// one thread per row: values and indices of its lane in its slice
__global__ __launch_bounds__(256) void k_xs_fill(const int64_t *rp, const int32_t *col, const double *val,
                                                 int64_t n, int64_t ns, const uint32_t *desc, const int32_t *soff,
                                                 const int32_t *coff, const int32_t *chunks, char *data) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= ns * 64) return;  // lanes past n in the last slice: padding (value 0, index 0)
    const int64_t s = r / 64, lane = r % 64, g = s / XS_SLICES;
    const int w = soff[s + 1] - soff[s];
    const uint32_t dsc = desc[s];
    char *blk = data + (int64_t)(dsc & 0x3fffffffu) * 128;
    double *vp = reinterpret_cast<double *>(blk);
    const int c0 = coff[g], nch = coff[g + 1] - c0;
    const int64_t e0 = r < n ? rp[r] : 0, len = r < n ? rp[r + 1] - e0 : 0;
    for (int t = 0; t < w; t++) {
        const bool in = t < len;
        const int32_t c = in ? col[e0 + t] : (len > 0 ? col[e0] : 0);
        vp[(int64_t)t * 64 + lane] = in ? val[e0 + t] : 0.0;
        if ((dsc >> 30) == 1) {
            const int32_t ch = c / XS_CH;
            int lo = 0, hi = nch - 1;  // the chunk's slot (present for every entry of an LDS slice)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (chunks[c0 + mid] < ch) lo = mid + 1;
                else hi = mid;
            }
            // padding of an empty row: slot 0, any in-range LDS entry
            const int32_t ix = (in || len > 0) ? lo * XS_CH + c % XS_CH : 0;
            reinterpret_cast<uint16_t *>(blk + (int64_t)w * 512)[(int64_t)t * 64 + lane] = (uint16_t)ix;
        } else {
            reinterpret_cast<int32_t *>(blk + (int64_t)w * 512)[(int64_t)t * 64 + lane] = c;
        }
    }
}

static bool xs_disabled() {
    static const bool off = [] {
        const char *e = getenv("FAMG_XS");
        return e && e[0] == '0';
    }();
    return off;
}

void xs_release(GpuCsr &m) {
    m.xs_data.release();
    m.xs_desc.release();
    m.xs_soff.release();
    m.xs_coff.release();
    m.xs_chunks.release();
    m.xs_groups = m.xs_bytes = m.xs_steps = m.xs_chunk_total = m.xs_escape_slices = m.xs_maxw = 0;
}

// Built for a single-segment matrix of >= XS_MIN_GROUPS groups (one workgroup
// per group: fewer leave CUs idle -- P_2 of the 256^3 cycle, 64 groups, ran 45 us
// against 21 us on SELL-64) whose SELL copy gathers (fewer than half of its
// slices with implicit columns) with fp64 values, when at most 1/16 of the
// slices escape.  True if built (the caller drops SELL).
constexpr int64_t XS_MIN_GROUPS = 512;

bool build_xs(GpuCsr &m, const std::vector<int64_t> &rp) {
    xs_release(m);
    if (xs_disabled() || g_spmv_format_policy != 0 || m.no_sellp || m.seg_rows.size() != 2 || !m.has_sell() ||
        m.sell_vbits != 0 || m.nrows < (XS_MIN_GROUPS - 1) * XS_ROWS + 1 || 2 * m.sell_mode_slices[0] >= m.nslices ||
        m.ncols >= (1 << 30))
        return false;
    const int64_t n = m.nrows, ns = (n + 63) / 64, ng = (ns + XS_SLICES - 1) / XS_SLICES;
    hipStream_t st = m.ctx->stream;
    std::vector<int32_t> col(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    std::vector<int32_t> w(ns), mode(ns);
    std::vector<std::vector<int32_t>> gch(ng);
    bool too_wide = false;
#pragma omp parallel for schedule(dynamic, 16) reduction(|| : too_wide)
    for (int64_t g = 0; g < ng; g++) {
        const int64_t r0 = g * XS_ROWS, r1 = std::min(n, r0 + XS_ROWS);
        std::vector<int32_t> ch;
        ch.reserve(rp[r1] - rp[r0]);
        for (int64_t e = rp[r0]; e < rp[r1]; e++) ch.push_back(col[e] / XS_CH);
        std::sort(ch.begin(), ch.end());
        // distinct chunks with their reference counts; keep the XS_MAXCH most referenced
        std::vector<std::pair<int32_t, int32_t>> cnt;  // (-count, chunk)
        for (size_t i = 0; i < ch.size();) {
            size_t j = i;
            while (j < ch.size() && ch[j] == ch[i]) j++;
            cnt.push_back({-(int32_t)(j - i), ch[i]});
            i = j;
        }
        if ((int)cnt.size() > XS_MAXCH) {
            std::nth_element(cnt.begin(), cnt.begin() + XS_MAXCH, cnt.end());
            cnt.resize(XS_MAXCH);
        }
        std::vector<int32_t> keep;
        for (auto &p : cnt) keep.push_back(p.second);
        std::sort(keep.begin(), keep.end());
        for (int64_t s = r0 / 64; s < (r1 + 63) / 64; s++) {
            int32_t ws = 0;
            bool esc = false;
            for (int64_t r = s * 64; r < std::min(n, s * 64 + 64); r++) {
                ws = std::max<int32_t>(ws, (int32_t)(rp[r + 1] - rp[r]));
                for (int64_t e = rp[r]; e < rp[r + 1] && !esc; e++)
                    esc = !std::binary_search(keep.begin(), keep.end(), col[e] / XS_CH);
            }
            if (ws > XS_MAX_W) too_wide = true;
            w[s] = std::max<int32_t>(ws, 1);  // an all-empty slice: one padding step (0.0 at index 0)
            mode[s] = esc ? 2 : 1;
        }
        if (keep.empty()) keep.push_back(0);
        gch[g] = std::move(keep);
    }
    if (too_wide) return false;
    int64_t esc = 0;
    for (int64_t s = 0; s < ns; s++) esc += mode[s] == 2;
    if (esc * 16 > ns) return false;
    std::vector<int32_t> soff(ns + 1, 0), coff(ng + 1, 0), chunks;
    std::vector<uint32_t> desc(ns);
    int64_t bytes = 0;
    for (int64_t s = 0; s < ns; s++) {
        if (bytes / 128 >= (int64_t(1) << 30)) return false;
        desc[s] = (uint32_t)(bytes / 128) | ((uint32_t)mode[s] << 30);
        bytes += ((int64_t)w[s] * 64 * (8 + (mode[s] == 1 ? 2 : 4)) + 127) / 128 * 128;
        soff[s + 1] = soff[s] + w[s];
    }
    for (int64_t g = 0; g < ng; g++) {
        chunks.insert(chunks.end(), gch[g].begin(), gch[g].end());
        coff[g + 1] = (int32_t)chunks.size();
    }
    m.xs_data.resize(std::max<int64_t>(128, bytes));  // every slice has >= 1 step: no load leaves it
    m.xs_desc.resize(ns);
    m.xs_soff.resize(ns + 1);
    m.xs_coff.resize(ng + 1);
    m.xs_chunks.resize(chunks.size());
    FAMG_CHECK_HIP(hipMemcpyAsync(m.xs_desc.get(), desc.data(), ns * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.xs_soff.get(), soff.data(), (ns + 1) * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.xs_coff.get(), coff.data(), (ng + 1) * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.xs_chunks.get(), chunks.data(), chunks.size() * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_xs_fill, dim3((unsigned)ceil_div(ns * 64, 256)), dim3(256), 0, st, m.rp64.get(), m.col.get(),
                       m.val.get(), n, ns, m.xs_desc.get(), m.xs_soff.get(), m.xs_coff.get(), m.xs_chunks.get(),
                       m.xs_data.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    m.xs_groups = ng;
    m.xs_bytes = bytes;
    m.xs_steps = soff[ns];
    m.xs_chunk_total = (int64_t)chunks.size();
    m.xs_escape_slices = esc;
    m.xs_maxw = *std::max_element(w.begin(), w.end());
    return true;
}

bool xs_supports(SpmvMode mode) { return mode != SPMV_SGS; }

#define FAMG_COMMA ,
void spmv_xs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s) {
    XsArgs a{m.xs_data.get(), m.xs_desc.get(), m.xs_soff.get(), m.xs_coff.get(), m.xs_chunks.get(),
             (int32_t)m.nrows, (int32_t)m.ncols, (int32_t)m.xs_groups, x, y, epi.b, epi.d, epi.dc, epi.dt};
    const dim3 grid((unsigned)m.xs_groups), block(XS_BS);
// T: the template arguments after the mode (empty, or ", NB")
#define FAMG_XS_LAUNCH(K, T)                                                          \
    switch (mode) {                                                                   \
    case SPMV_SET: K<SPMV_SET T><<<grid, block, 0, s>>>(a); break;                    \
    case SPMV_ADD: K<SPMV_ADD T><<<grid, block, 0, s>>>(a); break;                    \
    case SPMV_RESID: K<SPMV_RESID T><<<grid, block, 0, s>>>(a); break;                \
    case SPMV_JACOBI: K<SPMV_JACOBI T><<<grid, block, 0, s>>>(a); break;              \
    case SPMV_RESID0: K<SPMV_RESID0 T><<<grid, block, 0, s>>>(a); break;              \
    case SPMV_ADD0: K<SPMV_ADD0 T><<<grid, block, 0, s>>>(a); break;                  \
    default: fail(AMG_ERR_UNSUPPORTED, "x-staged SELL: unsupported SpMV epilogue"); \
    }
    const int64_t how = flag(FLAG_XS_PIPE);
    if (how >= 2 && m.xs_maxw <= 7) FAMG_XS_LAUNCH(spmv_xs_burst_kernel, FAMG_COMMA 7)
    else if (how >= 2) FAMG_XS_LAUNCH(spmv_xs_burst_kernel, FAMG_COMMA 8)
    else if (how == 1) FAMG_XS_LAUNCH(spmv_xs_pipe_kernel, )
    else FAMG_XS_LAUNCH(spmv_xs_kernel, )
#undef FAMG_XS_LAUNCH
#undef FAMG_COMMA
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
