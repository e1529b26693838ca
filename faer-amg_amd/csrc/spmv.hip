// spmv.hip -- fp64 CSR SpMV for gfx950 with fused V-cycle epilogues.
//
// Replaces the reference's CPU SpMV (ParSpmmOp, par_spmm.rs:98-133, and faer's
// SparseRowMat LinOp used at multigrid.rs:137-158) and fuses the vector work of
// Multigrid::cycle / smooth (multigrid.rs:341-350, 407-424) into its epilogue.
//
// Three kernels, chosen per matrix when it is finalized (csr_finalize):
//  * SELL-64 (short regular rows: the 7-pt fine level, P, R, A_1): one lane per
//    row, one wavefront per 64-row slice stored column-major -- every entry step
//    of a slice is one 512-B value / 256-B index access; no LDS, no barrier, no
//    row pointers; all loads of an <=8-entry chunk are issued before the
//    dependent x gathers.  Rows are summed sequentially (bit-identical to the
//    oracle).
//  * vector (very long rows, >= 256 entries on average: the densest Galerkin
//    operators near the coarsest level): one wavefront per row, lanes stride the row four 64-entry
//    steps at a time, shuffle-tree reduction.
//  * CSR-stream (everything else): blocks of <= 256 rows / <= 2048 entries
//    staged HBM -> LDS with 16-B non-temporal loads, L lanes per row.
// Workgroups are remapped so that each XCD (blocks b and b+8 share one) walks a
// contiguous slab of rows: a slab's x window (3 planes of a 7-pt operator,
// ~1.5 MB at 256^3) then stays in that XCD's 4 MB L2.
// A matrix may be cut into row segments (SGS colors, halo boundary/interior);
// every kernel can run one segment.
#include <algorithm>
#include <cstdlib>

#include "famg.hpp"

namespace famg {

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));

int g_spmv_format_policy = 0;
int g_alloc_policy = 1;
bool g_alloc_debug = [] {
    const char *e = getenv("FAMG_ALLOC_DEBUG");
    return e && e[0] == '1';
}();

constexpr int SPMV_BS = 256;
constexpr int SPMV_CAP = 2048;
constexpr int SELL_C = 64;
constexpr int SELL_MAX_W = 512;
constexpr int64_t SELL_MIN_ROWS = 65536;
constexpr int VECTOR_MIN_AVG = 256;

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, idx = b >> 3;
    return x * q + min(x, r) + idx;
}

struct Epi {
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const int32_t *perm;
};

// Operands of the epilogue that do not depend on the row sum are fetched
// before the row's loads are issued.
template <int MODE> struct EpiOps {
    double xr = 0.0, br = 0.0, dr = 0.0, yr = 0.0;
    int i = 0;
    __device__ __forceinline__ void load(const Epi &a, int row) {
        i = row;
        if constexpr (MODE == SPMV_SGS) i = a.perm[row];
        if constexpr (MODE == SPMV_JACOBI || MODE == SPMV_SGS) { xr = a.x[i]; br = a.b[i]; dr = a.d[row]; }
        if constexpr (MODE == SPMV_RESID) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
    }
    __device__ __forceinline__ void store(const Epi &a, double acc) const {
        if constexpr (MODE == SPMV_SET) a.y[i] = acc;
        else if constexpr (MODE == SPMV_ADD) a.y[i] = yr + acc;
        else if constexpr (MODE == SPMV_RESID) a.y[i] = br - acc;
        else a.y[i] = xr + dr * (br - acc);  // JACOBI, SGS
    }
};

// ---------------------------------------------------------------- CSR-stream

struct StreamArgs {
    const int32_t *rowptr;
    const int32_t *col;
    const double *val;
    const int32_t *sched;
    int32_t nblocks;
    Epi e;
};

template <int MODE>
__global__ __launch_bounds__(SPMV_BS) void spmv_stream_kernel(StreamArgs a) {
    __shared__ __attribute__((aligned(16))) double sval[SPMV_CAP + 2];
    __shared__ __attribute__((aligned(16))) int32_t scol[SPMV_CAP + 4];
    __shared__ double sred[SPMV_BS / 64];

    const int blk = xcd_remap(blockIdx.x, a.nblocks);
    const int r0 = a.sched[blk], r1 = a.sched[blk + 1];
    const int e0 = a.rowptr[r0], e1 = a.rowptr[r1];
    const int tid = threadIdx.x;
    const int nnz = e1 - e0;

    if (nnz > SPMV_CAP) {  // one long row (r1 == r0 + 1): the whole workgroup reduces it
        double acc = 0.0;
        for (int k = e0 + tid; k < e1; k += SPMV_BS) acc = fma(a.val[k], a.e.x[a.col[k]], acc);
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if ((tid & 63) == 0) sred[tid >> 6] = acc;
        __syncthreads();
        if (tid == 0) {
            double s = sred[0];
            for (int w = 1; w < SPMV_BS / 64; w++) s += sred[w];
            EpiOps<MODE> ep;
            ep.load(a.e, r0);
            ep.store(a.e, s);
        }
        return;
    }
    const int nrows = r1 - r0;
    int L = 1;
    while (L < 64 && 2 * L * nrows <= SPMV_BS) L <<= 1;
    const int rl = tid / L;
    const int sub = tid & (L - 1);
    EpiOps<MODE> ep;
    if (rl < nrows && sub == 0) ep.load(a.e, r0 + rl);

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

    const int vo = e0 - bv, co = e0 - bc;
    double acc = 0.0;
    if (rl < nrows) {
        const int rs = a.rowptr[r0 + rl] - e0;
        const int re = a.rowptr[r0 + rl + 1] - e0;
        for (int k = rs + sub; k < re; k += L) acc = fma(sval[vo + k], a.e.x[scol[co + k]], acc);
    }
    for (int off = L >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (rl < nrows && sub == 0) ep.store(a.e, acc);
}

// ------------------------------------------------------------------- SELL-64

// Interleaved slice storage: entry step k of a slice is one 768-B record
// [64 fp64 values | 64 int32 columns], so a wavefront streams a single
// contiguous region and a matrix needs one allocation.
constexpr int SELL_STEP_BYTES = SELL_C * 12;
constexpr int SELL_V_STRIDE = SELL_STEP_BYTES / 8;   // doubles per step
constexpr int SELL_C_STRIDE = SELL_STEP_BYTES / 4;   // int32 per step

struct SellArgs {
    const int32_t *off;   // entry offset of each slice (nslices+1)
    const int32_t *row0;  // first row of each slice (nslices+1; slices tile the rows)
    const char *data;     // interleaved records, slice s at byte 12 * off[s]
    int32_t slice0, nslices;
    Epi e;
};

template <int U>
__device__ __forceinline__ void sell_chunk(const double *__restrict__ v, const int32_t *__restrict__ c,
                                           const double *__restrict__ x, double &acc) {
    double vv[U];
    int32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        vv[u] = __builtin_nontemporal_load(v + u * SELL_V_STRIDE);
        cc[u] = __builtin_nontemporal_load(c + u * SELL_C_STRIDE);
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
    const int sl = blk * 4 + (threadIdx.x >> 6);
    if (sl >= a.nslices) return;
    const int slice = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int row = a.row0[slice] + lane;
    const bool live = row < a.row0[slice + 1];
    EpiOps<MODE> ep;
    if (live) ep.load(a.e, row);
    const int o0 = a.off[slice];
    const int w = (a.off[slice + 1] - o0) >> 6;
    const char *base = a.data + (int64_t)o0 * 12;
    const double *v = reinterpret_cast<const double *>(base) + lane;
    const int32_t *c = reinterpret_cast<const int32_t *>(base + SELL_C * 8) + lane;
    const double *x = a.e.x;
    double acc = 0.0;
    int k = 0;
    for (; k + 8 <= w; k += 8) sell_chunk<8>(v + k * SELL_V_STRIDE, c + k * SELL_C_STRIDE, x, acc);
    v += k * SELL_V_STRIDE;
    c += k * SELL_C_STRIDE;
    switch (w - k) {
    case 1: sell_chunk<1>(v, c, x, acc); break;
    case 2: sell_chunk<2>(v, c, x, acc); break;
    case 3: sell_chunk<3>(v, c, x, acc); break;
    case 4: sell_chunk<4>(v, c, x, acc); break;
    case 5: sell_chunk<5>(v, c, x, acc); break;
    case 6: sell_chunk<6>(v, c, x, acc); break;
    case 7: sell_chunk<7>(v, c, x, acc); break;
    default: break;
    }
    if (live) ep.store(a.e, acc);
}

// --------------------------------------------------------------------- vector

struct VecArgs {
    const int32_t *rowptr;
    const int32_t *col;
    const double *val;
    int32_t row_begin, nrows;
    Epi e;
};

template <int MODE>
__global__ __launch_bounds__(256) void spmv_vector_kernel(VecArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int w = blk * 4 + (threadIdx.x >> 6);
    if (w >= a.nrows) return;
    const int row = a.row_begin + w;
    const int lane = threadIdx.x & 63;
    EpiOps<MODE> ep;
    if (lane == 0) ep.load(a.e, row);
    const int e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
    const double *__restrict__ val = a.val;
    const int32_t *__restrict__ col = a.col;
    const double *__restrict__ x = a.e.x;
    double acc = 0.0;
    int k = e0 + lane;
    for (; k + 3 * 64 < e1; k += 4 * 64) {
        double vv[4];
        int32_t cc[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            vv[u] = __builtin_nontemporal_load(val + k + 64 * u);
            cc[u] = __builtin_nontemporal_load(col + k + 64 * u);
        }
        double xx[4];
#pragma unroll
        for (int u = 0; u < 4; u++) xx[u] = x[cc[u]];
#pragma unroll
        for (int u = 0; u < 4; u++) acc = fma(vv[u], xx[u], acc);
    }
    for (; k < e1; k += 64) acc = fma(__builtin_nontemporal_load(val + k), x[__builtin_nontemporal_load(col + k)], acc);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) ep.store(a.e, acc);
}

// ------------------------------------------------------------ host: storage

// Greedy blocks of <= SPMV_BS rows and <= SPMV_CAP nonzeros per segment; a row
// longer than SPMV_CAP is a block of its own.
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

__global__ void k_sell_fill(const int64_t *rp, const int32_t *col, const double *val,
                            const int32_t *off, const int32_t *row0, int64_t nslices, char *data) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nslices * SELL_C) return;
    const int64_t s = t / SELL_C, lane = t % SELL_C;
    const int64_t r = row0[s] + lane;
    const bool live = r < row0[s + 1];
    const int64_t len = live ? rp[r + 1] - rp[r] : 0;
    const int64_t base = live ? rp[r] : 0;
    const int w = (off[s + 1] - off[s]) / SELL_C;
    const int32_t cpad = len > 0 ? col[base + len - 1] : 0;
    char *slice = data + (int64_t)off[s] * 12;
    for (int k = 0; k < w; k++) {
        double *sv = reinterpret_cast<double *>(slice + (int64_t)k * SELL_STEP_BYTES) + lane;
        int32_t *sc = reinterpret_cast<int32_t *>(slice + (int64_t)k * SELL_STEP_BYTES + SELL_C * 8) + lane;
        if (k < len) { *sc = col[base + k]; *sv = val[base + k]; }
        else { *sc = cpad; *sv = 0.0; }
    }
}

void build_sell(GpuCsr &m, const std::vector<int64_t> &rp) {
    m.sell_off.release();
    m.sell_row0.release();
    m.sell_data.release();
    m.nslices = m.sell_padded = 0;
    m.seg_slc.clear();
    const int pol = g_spmv_format_policy;
    if (pol == 1 || pol == 3 || m.nrows == 0 || m.nnz == 0) return;
    std::vector<int32_t> off{0}, row0;
    std::vector<int64_t> seg_slc{0};
    int64_t padded = 0, maxw = 0;
    for (size_t g = 0; g + 1 < m.seg_rows.size(); g++) {
        for (int64_t r0 = m.seg_rows[g]; r0 < m.seg_rows[g + 1]; r0 += SELL_C) {
            const int64_t r1 = std::min<int64_t>(m.seg_rows[g + 1], r0 + SELL_C);
            int64_t w = 0;
            for (int64_t r = r0; r < r1; r++) w = std::max<int64_t>(w, rp[r + 1] - rp[r]);
            maxw = std::max(maxw, w);
            padded += w * SELL_C;
            if (padded >= (int64_t(1) << 31)) return;
            off.push_back(static_cast<int32_t>(padded));
            row0.push_back(static_cast<int32_t>(r0));
        }
        seg_slc.push_back(static_cast<int64_t>(row0.size()));
    }
    row0.push_back(static_cast<int32_t>(m.nrows));
    // auto: SELL pays when there are enough slices to fill the chip (>= 1024
    // slices = 64K rows) and padding is modest; measured on the 256^3 hierarchy
    // (scripts/ab_levels.py) it beats CSR-stream up to ~170-entry rows.
    const bool ok = pol == 2 ? maxw <= 256
                             : (maxw <= SELL_MAX_W && padded * 100 <= m.nnz * 125 &&
                                (m.nrows >= SELL_MIN_ROWS || maxw <= 16));
    if (!ok) return;
    const int64_t ns = static_cast<int64_t>(off.size()) - 1;
    hipStream_t s = m.ctx->stream;
    m.sell_off.resize(ns + 1);
    m.sell_row0.resize(ns + 1);
    m.sell_data.resize(padded * 12);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_off.get(), off.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_row0.get(), row0.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_sell_fill, dim3((unsigned)ceil_div(ns * SELL_C, 256)), dim3(256), 0, s,
                       m.rp64.get(), m.col.get(), m.val.get(), m.sell_off.get(), m.sell_row0.get(), ns,
                       m.sell_data.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.nslices = ns;
    m.sell_padded = padded;
    m.seg_slc = seg_slc;
}

void choose_kernel(GpuCsr &m) {
    if (m.has_sell()) m.kernel = SPMV_KERNEL_SELL;
    else if (g_spmv_format_policy == 3 ||
             (g_spmv_format_policy == 0 && m.nrows > 0 && m.nnz >= VECTOR_MIN_AVG * m.nrows))
        m.kernel = SPMV_KERNEL_VECTOR;
    else m.kernel = SPMV_KERNEL_STREAM;
}

// ------------------------------------------------------------------ dispatch

#define FAMG_LAUNCH_MODES(KERNEL, grid, block, s, args)                                       \
    switch (mode) {                                                                           \
    case SPMV_SET: hipLaunchKernelGGL(KERNEL<SPMV_SET>, grid, block, 0, s, args); break;      \
    case SPMV_ADD: hipLaunchKernelGGL(KERNEL<SPMV_ADD>, grid, block, 0, s, args); break;      \
    case SPMV_RESID: hipLaunchKernelGGL(KERNEL<SPMV_RESID>, grid, block, 0, s, args); break;  \
    case SPMV_JACOBI: hipLaunchKernelGGL(KERNEL<SPMV_JACOBI>, grid, block, 0, s, args); break; \
    case SPMV_SGS: hipLaunchKernelGGL(KERNEL<SPMV_SGS>, grid, block, 0, s, args); break;      \
    }

void spmv(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
          hipStream_t s, int64_t seg) {
    FAMG_REQUIRE(m.spmv_ready(), AMG_ERR_UNSUPPORTED, "SpMV needs nnz < 2^31 (32-bit row pointers)");
    FAMG_REQUIRE(seg < (int64_t)m.seg_rows.size() - 1, AMG_ERR_INVALID, "SpMV segment out of range");
    FAMG_REQUIRE(mode != SPMV_SGS || epi.perm, AMG_ERR_INVALID, "SGS mode needs a permutation");
    Epi e{x, y, epi.b, epi.d, epi.perm};
    const dim3 block(256);
    if (m.kernel == SPMV_KERNEL_SELL) {
        const int64_t s0 = seg < 0 ? 0 : m.seg_slc[seg];
        const int64_t s1 = seg < 0 ? m.nslices : m.seg_slc[seg + 1];
        if (s1 <= s0) return;
        SellArgs a{m.sell_off.get(), m.sell_row0.get(), m.sell_data.get(), (int32_t)s0,
                   (int32_t)(s1 - s0), e};
        const dim3 grid((unsigned)ceil_div(s1 - s0, 4));
        FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a)
    } else if (m.kernel == SPMV_KERNEL_VECTOR) {
        const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg];
        const int64_t r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
        if (r1 <= r0) return;
        VecArgs a{m.rp32.get(), m.col.get(), m.val.get(), (int32_t)r0, (int32_t)(r1 - r0), e};
        const dim3 grid((unsigned)ceil_div(r1 - r0, 4));
        FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a)
    } else {
        const int64_t b0 = seg < 0 ? 0 : m.seg_blk[seg];
        const int64_t b1 = seg < 0 ? m.nblocks : m.seg_blk[seg + 1];
        if (b1 <= b0) return;
        StreamArgs a{m.rp32.get(), m.col.get(), m.val.get(), m.sched.get() + b0, (int32_t)(b1 - b0), e};
        const dim3 grid((unsigned)(b1 - b0));
        FAMG_LAUNCH_MODES(spmv_stream_kernel, grid, block, s, a)
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
