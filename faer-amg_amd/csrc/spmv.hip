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

#include <cstring>

namespace famg {

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));

int g_spmv_format_policy = 0;
int g_value_codes = 1;
int g_alloc_policy = 0;
int g_alloc_experiment = [] {
    const char *e = getenv("FAMG_ALLOC_EXPERIMENT");
    return e ? atoi(e) : 0;
}();
bool g_alloc_debug = [] {
    const char *e = getenv("FAMG_ALLOC_DEBUG");
    return e && e[0] == '1';
}();
// DIA storage: FAMG_DIA_NT=1 streams the epilogue operands (b, d, y) with
// non-temporal accesses (A/B switch; results are bitwise equal).
// FAMG_DIA_BANDS=0 turns the 2.5-D (plane-band per XCD) block order off
static bool dia_bands() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_BANDS");
        return !(e && e[0] == '0');
    }();
    return on;
}
static bool dia_nt() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_NT");
        return e && e[0] == '1';
    }();
    return on;
}

constexpr int SPMV_BS = 256;
constexpr int SPMV_CAP = 2048;
constexpr int SELL_C = 64;
constexpr int SELL_MAX_W = 512;
constexpr int64_t SELL_MIN_ROWS = 65536;
constexpr int VECTOR_MIN_AVG = 256;
// rows at least this long on average take the wave-per-row kernel; A/B switch
// FAMG_VECTOR_MIN_AVG (lower values replace SELL on A_2: measured 2.7x slower)
static int64_t vec_min_avg() {
    static const int64_t v = [] {
        const char *e = getenv("FAMG_VECTOR_MIN_AVG");
        const int64_t x = e ? atoll(e) : 0;
        return x > 0 ? x : (int64_t)VECTOR_MIN_AVG;
    }();
    return v;
}
constexpr int64_t SELL_PAIR_MIN_SLICES = 1;  // pairing paid on every level measured (A_2: 55 vs 60 us)


struct Epi {
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const int32_t *perm;
    const uint8_t *dc;  // JACOBI: d[i] = dt[dc[i]] when set (8-bit codes of the diagonal)
    const double *dt;
    double dk;          // d when it is one value (the constant-diagonal epilogues)
};

// Operands of the epilogue that do not depend on the row sum are fetched
// before the row's loads are issued.
template <int MODE> struct EpiOps {
    double xr = 0.0, br = 0.0, dr = 0.0, yr = 0.0;
    int i = 0;
    __device__ __forceinline__ void load(const Epi &a, int row) {
        i = row;
        if constexpr (MODE == SPMV_SGS) i = a.perm[row];
        if constexpr (MODE == SPMV_JACOBI || MODE == SPMV_SGS) {
            xr = a.x[i];
            br = a.b[i];
            dr = (MODE == SPMV_JACOBI && a.dc) ? a.dt[a.dc[row]] : a.d[row];
        }
        if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
        if constexpr (MODE == SPMV_ADD0) yr = (a.dc ? a.dt[a.dc[row]] : a.d[row]) * a.b[row];
    }
    __device__ __forceinline__ void store(const Epi &a, double acc) const {
        if constexpr (MODE == SPMV_SET) a.y[i] = acc;
        else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[i] = yr + acc;
        else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[i] = br - acc;
        else a.y[i] = xr + dr * (br - acc);  // JACOBI, SGS
    }
};

// The x operand of a row sum: x[c], or for RESID0 the zero-guess Jacobi
// iterate d[c]*x[c] -- the same rounded product vec_mul would have stored.
template <int MODE> __device__ __forceinline__ double gx(const Epi &e, int c) {
    if constexpr (MODE == SPMV_RESID0) return e.d[c] * e.x[c];
    else return e.x[c];
}

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
        for (int k = e0 + tid; k < e1; k += SPMV_BS) acc = fma(a.val[k], gx<MODE>(a.e, a.col[k]), acc);
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
        for (int k = rs + sub; k < re; k += L) acc = fma(sval[vo + k], gx<MODE>(a.e, scol[co + k]), acc);
    }
    for (int off = L >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (rl < nrows && sub == 0) ep.store(a.e, acc);
}

// ------------------------------------------------------------------- SELL-64
//
// Slice s = up to 64 consecutive rows, one lane per row, w_s entry steps.  The
// slice's block in sell_data is [w_s x 64 fp64 values | column block], the
// column of lane l at step t given by the slice's column mode:
//   0 implicit  col = base[t] + l                    (0 B/entry)
//   1 u16       col = base[t] + d16(t, l)            (2 B/entry)
//   2 i32       col = c32(t, l)                      (4 B/entry)
// Steps are either the k-th stored entry of every row ("plain") or, when it is
// cheaper, the sorted union of the slice's column offsets col - row
// ("aligned"; a stencil row then reads x[row + offset] for offset t: mode 0
// and coalesced x loads).  A row without an entry at a step holds 0.0 at an
// in-range column, so every row is still summed in its stored (ascending
// column) order with fma, interleaved with exact +0 terms: bit-identical to the
// CSR kernels for finite x.
//
// Element order inside a block (values, and the u16/i32 column block alike):
// steps are stored in PAIRS -- step t < 2*floor(w/2) of lane l at element
// (t & ~1)*64 + 2l + (t & 1) -- so one 16-B load per lane brings the values of
// two steps (4 B / 8 B for two compressed columns); an odd last step is stored
// plainly at t*64 + l.  Streamed with 8-B non-temporal loads the values ran at
// roughly 0.54-0.70x the 16-B rate (MI355X_MICROARCH.md, L2-served loads).
// `sell_paired = false` keeps one 512-B row per step (A/B switch,
// FAMG_SELL_LAYOUT=step at build time).
constexpr int SELL_VAL_STEP = SELL_C * 8;  // bytes of values per step

typedef int32_t i32x2_t __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ int64_t sell_elem(int t, int w, int lane, bool paired) {
    if (paired && (t | 1) < w) return (int64_t)(t & ~1) * SELL_C + 2 * lane + (t & 1);
    return (int64_t)t * SELL_C + lane;
}

struct SellArgs {
    const int32_t *row0;   // nslices+1 (slices tile the rows)
    const int32_t *soff;   // nslices+1 step offsets
    const uint32_t *desc;  // block offset / 128 | mode << 30
    const int32_t *base;   // one per step
    const char *data;
    int32_t slice0, nslices;
    Epi e;
    const double *vtab;  // value table (code widths 4 / 8 / 16)
    int32_t ntab;
    int32_t spw;  // slices per wave (value codes: 2 on large matrices, else 1)
};

// ---- one step per 512-B row (sell_paired = false)

template <int MODE, int CM, int U>
__device__ __forceinline__ void sell_chunk(const double *__restrict__ v, const void *__restrict__ ix,
                                           const int32_t *__restrict__ bs, int lane, const Epi &e, double &acc) {
    double vv[U];
    int32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        vv[u] = __builtin_nontemporal_load(v + u * SELL_C);
        if constexpr (CM == 0) cc[u] = bs[u] + lane;
        else if constexpr (CM == 1)
            cc[u] = bs[u] + (int32_t)__builtin_nontemporal_load(static_cast<const uint16_t *>(ix) + u * SELL_C);
        else cc[u] = __builtin_nontemporal_load(static_cast<const int32_t *>(ix) + u * SELL_C);
    }
    double xx[U];
#pragma unroll
    for (int u = 0; u < U; u++) xx[u] = gx<MODE>(e, cc[u]);
#pragma unroll
    for (int u = 0; u < U; u++) acc = fma(vv[u], xx[u], acc);
}

template <int MODE, int CM>
__device__ __forceinline__ double sell_walk_steps(const char *blkp, const int32_t *bs, int w, int lane,
                                                  const Epi &e) {
    constexpr int IB = CM == 0 ? 0 : CM == 1 ? 2 : 4;  // index bytes per entry
    const double *v = reinterpret_cast<const double *>(blkp) + lane;
    const char *ix = blkp + (int64_t)w * SELL_VAL_STEP + lane * IB;
    double acc = 0.0;
    int k = 0;
    for (; k + 8 <= w; k += 8)
        sell_chunk<MODE, CM, 8>(v + k * SELL_C, ix + (int64_t)k * SELL_C * IB, bs + k, lane, e, acc);
    v += k * SELL_C;
    ix += (int64_t)k * SELL_C * IB;
    bs += k;
    switch (w - k) {
    case 1: sell_chunk<MODE, CM, 1>(v, ix, bs, lane, e, acc); break;
    case 2: sell_chunk<MODE, CM, 2>(v, ix, bs, lane, e, acc); break;
    case 3: sell_chunk<MODE, CM, 3>(v, ix, bs, lane, e, acc); break;
    case 4: sell_chunk<MODE, CM, 4>(v, ix, bs, lane, e, acc); break;
    case 5: sell_chunk<MODE, CM, 5>(v, ix, bs, lane, e, acc); break;
    case 6: sell_chunk<MODE, CM, 6>(v, ix, bs, lane, e, acc); break;
    case 7: sell_chunk<MODE, CM, 7>(v, ix, bs, lane, e, acc); break;
    default: break;
    }
    return acc;
}

// ---- step pairs (sell_paired = true)

// UP step pairs starting at pair p0, plus the odd last step when TAIL; every
// load of the group is issued before the dependent x gathers, and the row sum
// still runs over t ascending.
template <int MODE, int CM, int UP, bool TAIL>
__device__ __forceinline__ void sell_pairs(const char *__restrict__ blkp, int w, int p0,
                                           const int32_t *__restrict__ bs, int lane, const Epi &e, double &acc) {
    constexpr int NS = 2 * UP + (TAIL ? 1 : 0);
    double vv[NS];
    int32_t cc[NS];
    const char *ixb = blkp + (int64_t)w * SELL_VAL_STEP;
#pragma unroll
    for (int u = 0; u < UP; u++) {
        const int64_t q = (int64_t)(p0 + u) * SELL_C + lane;  // 2-element unit of this lane
        const dbl2_t v = __builtin_nontemporal_load(reinterpret_cast<const dbl2_t *>(blkp) + q);
        vv[2 * u] = v.x;
        vv[2 * u + 1] = v.y;
        const int t = 2 * (p0 + u);
        if constexpr (CM == 0) {
            cc[2 * u] = bs[t] + lane;
            cc[2 * u + 1] = bs[t + 1] + lane;
        } else if constexpr (CM == 1) {
            const uint32_t d = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(ixb) + q);
            cc[2 * u] = bs[t] + (int32_t)(d & 0xffffu);
            cc[2 * u + 1] = bs[t + 1] + (int32_t)(d >> 16);
        } else {
            const i32x2_t d = __builtin_nontemporal_load(reinterpret_cast<const i32x2_t *>(ixb) + q);
            cc[2 * u] = d.x;
            cc[2 * u + 1] = d.y;
        }
    }
    if constexpr (TAIL) {
        const int t = w - 1;
        const int64_t el = (int64_t)t * SELL_C + lane;
        vv[NS - 1] = __builtin_nontemporal_load(reinterpret_cast<const double *>(blkp) + el);
        if constexpr (CM == 0) cc[NS - 1] = bs[t] + lane;
        else if constexpr (CM == 1)
            cc[NS - 1] = bs[t] + (int32_t)__builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(ixb) + el);
        else cc[NS - 1] = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(ixb) + el);
    }
    double xx[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) xx[u] = gx<MODE>(e, cc[u]);
#pragma unroll
    for (int u = 0; u < NS; u++) acc = fma(vv[u], xx[u], acc);
}

template <int MODE, int CM>
__device__ __forceinline__ double sell_walk_pairs(const char *blkp, const int32_t *bs, int w, int lane,
                                                  const Epi &e) {
    double acc = 0.0;
    const int np = w >> 1;
    int p = 0;
    for (; p + 4 <= np; p += 4) sell_pairs<MODE, CM, 4, false>(blkp, w, p, bs, lane, e, acc);
    switch (2 * (np - p) + (w & 1)) {
    case 1: sell_pairs<MODE, CM, 0, true>(blkp, w, p, bs, lane, e, acc); break;
    case 2: sell_pairs<MODE, CM, 1, false>(blkp, w, p, bs, lane, e, acc); break;
    case 3: sell_pairs<MODE, CM, 1, true>(blkp, w, p, bs, lane, e, acc); break;
    case 4: sell_pairs<MODE, CM, 2, false>(blkp, w, p, bs, lane, e, acc); break;
    case 5: sell_pairs<MODE, CM, 2, true>(blkp, w, p, bs, lane, e, acc); break;
    case 6: sell_pairs<MODE, CM, 3, false>(blkp, w, p, bs, lane, e, acc); break;
    case 7: sell_pairs<MODE, CM, 3, true>(blkp, w, p, bs, lane, e, acc); break;
    default: break;
    }
    return acc;
}

// ---- value codes (sell_vbits = 4, 8 or 16)
//
// A matrix whose stored values take at most 16 / 256 / 65536 distinct fp64 bit
// patterns (the padding's +0.0 included) stores a 4 / 8 / 16-bit code per
// entry into a per-matrix table sorted by bit pattern instead of the value
// (index/value compression in the manner of CSR-VI).  The 8 codes of steps
// 8g..8g+7 of one lane form one 4 / 8 / 16-B unit at g*64 + lane.  Column
// blocks (u16 / i32) use the same grouping: step t of lane l at element
// 8g*64 + r_g*l + (t - 8g), r_g = min(8, w - 8g), so a full group is one (u16)
// or two (i32) 16-B loads per lane.  Tables of <= 256 entries are staged in
// LDS per workgroup, 16-bit tables are read through the caches.  A decoded
// value is the stored value bit for bit, so every row sum is unchanged.
__host__ __device__ __forceinline__ int sell_code_bytes(int vb) { return vb == 4 ? 4 : vb == 8 ? 8 : 16; }

__host__ __device__ __forceinline__ int64_t sell_value_bytes(int64_t w, int vb) {
    return vb ? ((w + 7) >> 3) * SELL_C * sell_code_bytes(vb) : w * SELL_VAL_STEP;
}

__host__ __device__ __forceinline__ int64_t sell_group_elem(int t, int w, int lane) {
    const int g0 = t & ~7;
    const int r = w - g0 < 8 ? w - g0 : 8;
    return (int64_t)g0 * SELL_C + r * lane + (t & 7);
}

template <int VB>
__device__ __forceinline__ void sell_load_codes(const char *__restrict__ blkp, int g, int lane, uint32_t (&q)[4]) {
    const int64_t unit = (int64_t)g * SELL_C + lane;
    if constexpr (VB == 4) {
        q[0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(blkp) + unit);
    } else if constexpr (VB == 8) {
        const i32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x2_t *>(blkp) + unit);
        q[0] = (uint32_t)v.x;
        q[1] = (uint32_t)v.y;
    } else {
        const i32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t *>(blkp) + unit);
        q[0] = (uint32_t)v.x;
        q[1] = (uint32_t)v.y;
        q[2] = (uint32_t)v.z;
        q[3] = (uint32_t)v.w;
    }
}

template <int VB> __device__ __forceinline__ int sell_code(const uint32_t (&q)[4], int u) {
    if constexpr (VB == 4) return (int)((q[0] >> (4 * u)) & 15u);
    else if constexpr (VB == 8) return (int)((q[u >> 2] >> (8 * (u & 3))) & 255u);
    else return (int)((q[u >> 1] >> (16 * (u & 1))) & 0xffffu);
}

// Columns of the R (<= 8) steps of group g (first step t0 = 8g).
template <int CM, int R>
__device__ __forceinline__ void sell_group_cols(const char *__restrict__ ixb, const int32_t *__restrict__ bs, int t0,
                                                int lane, int32_t (&cc)[R]) {
    if constexpr (CM == 0) {
#pragma unroll
        for (int u = 0; u < R; u++) cc[u] = bs[t0 + u] + lane;
    } else if constexpr (R == 8) {
        const int64_t el = (int64_t)t0 * SELL_C + 8 * lane;
        if constexpr (CM == 1) {
            const i32x4_t d = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t *>(ixb + 2 * el));
#pragma unroll
            for (int u = 0; u < 4; u++) {
                cc[2 * u] = bs[t0 + 2 * u] + (int32_t)((uint32_t)d[u] & 0xffffu);
                cc[2 * u + 1] = bs[t0 + 2 * u + 1] + (int32_t)((uint32_t)d[u] >> 16);
            }
        } else {
            const i32x4_t *p = reinterpret_cast<const i32x4_t *>(ixb + 4 * el);
            const i32x4_t d0 = __builtin_nontemporal_load(p);
            const i32x4_t d1 = __builtin_nontemporal_load(p + 1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                cc[u] = d0[u];
                cc[4 + u] = d1[u];
            }
        }
    } else {
        const int64_t el = (int64_t)t0 * SELL_C + R * lane;
#pragma unroll
        for (int u = 0; u < R; u++) {
            if constexpr (CM == 1)
                cc[u] = bs[t0 + u] +
                        (int32_t)__builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(ixb) + el + u);
            else cc[u] = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(ixb) + el + u);
        }
    }
}

// R (<= 8) steps of group g: every load of the group is issued before the
// dependent x gathers; the row sum runs over t ascending.
template <int MODE, int CM, int VB, int R>
__device__ __forceinline__ void sellc_group(const char *__restrict__ blkp, const char *__restrict__ ixb, int g,
                                            const int32_t *__restrict__ bs, int lane, const double *tab,
                                            const Epi &e, double &acc) {
    uint32_t q[4];
    sell_load_codes<VB>(blkp, g, lane, q);
    int32_t cc[R];
    sell_group_cols<CM, R>(ixb, bs, 8 * g, lane, cc);
    double xx[R];
#pragma unroll
    for (int u = 0; u < R; u++) xx[u] = gx<MODE>(e, cc[u]);
#pragma unroll
    for (int u = 0; u < R; u++) acc = fma(tab[sell_code<VB>(q, u)], xx[u], acc);
}

// The same for two slices of equal width and column mode in lockstep: the
// loads of both slices are in flight together (a codes slice streams few
// bytes, so one slice per wave leaves the memory system latency-bound).
template <int MODE, int CM, int VB, int R>
__device__ __forceinline__ void sellc_group2(const char *__restrict__ ba, const char *__restrict__ bb,
                                             const char *__restrict__ ia, const char *__restrict__ ib, int g,
                                             const int32_t *__restrict__ sa, const int32_t *__restrict__ sb,
                                             int lane, const double *tab, const Epi &e, double &acca,
                                             double &accb) {
    uint32_t qa[4], qb[4];
    sell_load_codes<VB>(ba, g, lane, qa);
    sell_load_codes<VB>(bb, g, lane, qb);
    int32_t ca[R], cb[R];
    sell_group_cols<CM, R>(ia, sa, 8 * g, lane, ca);
    sell_group_cols<CM, R>(ib, sb, 8 * g, lane, cb);
    double xa[R], xb[R];
#pragma unroll
    for (int u = 0; u < R; u++) {
        xa[u] = gx<MODE>(e, ca[u]);
        xb[u] = gx<MODE>(e, cb[u]);
    }
#pragma unroll
    for (int u = 0; u < R; u++) acca = fma(tab[sell_code<VB>(qa, u)], xa[u], acca);
#pragma unroll
    for (int u = 0; u < R; u++) accb = fma(tab[sell_code<VB>(qb, u)], xb[u], accb);
}

template <int MODE, int CM, int VB>
__device__ __forceinline__ void sellc_walk2(const char *ba, const char *bb, const int32_t *sa, const int32_t *sb,
                                            int w, int lane, const double *tab, const Epi &e, double &acca,
                                            double &accb) {
    const int ng = (w + 7) >> 3;
    const char *ia = ba + (int64_t)ng * SELL_C * sell_code_bytes(VB);
    const char *ib = bb + (int64_t)ng * SELL_C * sell_code_bytes(VB);
    acca = 0.0;
    accb = 0.0;
    const int full = w >> 3;
    for (int g = 0; g < full; g++) sellc_group2<MODE, CM, VB, 8>(ba, bb, ia, ib, g, sa, sb, lane, tab, e, acca, accb);
    switch (w & 7) {
    case 1: sellc_group2<MODE, CM, VB, 1>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 2: sellc_group2<MODE, CM, VB, 2>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 3: sellc_group2<MODE, CM, VB, 3>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 4: sellc_group2<MODE, CM, VB, 4>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 5: sellc_group2<MODE, CM, VB, 5>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 6: sellc_group2<MODE, CM, VB, 6>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    case 7: sellc_group2<MODE, CM, VB, 7>(ba, bb, ia, ib, full, sa, sb, lane, tab, e, acca, accb); break;
    default: break;
    }
}

template <int MODE, int CM, int VB>
__device__ __forceinline__ double sellc_walk(const char *blkp, const int32_t *bs, int w, int lane, const double *tab,
                                             const Epi &e) {
    const int ng = (w + 7) >> 3;
    const char *ixb = blkp + (int64_t)ng * SELL_C * sell_code_bytes(VB);
    double acc = 0.0;
    const int full = w >> 3;
    // two groups' loads in one block, except RESID0 (two gathers per entry
    // already; the doubled footprint cost occupancy)
    constexpr int UNR = MODE == SPMV_RESID0 ? 1 : 2;
#pragma unroll UNR
    for (int g = 0; g < full; g++) sellc_group<MODE, CM, VB, 8>(blkp, ixb, g, bs, lane, tab, e, acc);
    switch (w & 7) {
    case 1: sellc_group<MODE, CM, VB, 1>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 2: sellc_group<MODE, CM, VB, 2>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 3: sellc_group<MODE, CM, VB, 3>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 4: sellc_group<MODE, CM, VB, 4>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 5: sellc_group<MODE, CM, VB, 5>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 6: sellc_group<MODE, CM, VB, 6>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    case 7: sellc_group<MODE, CM, VB, 7>(blkp, ixb, full, bs, lane, tab, e, acc); break;
    default: break;
    }
    return acc;
}

// ---- lockstep pair, two adjacent rows per lane
//
// Lanes 0-31 take rows 2h, 2h+1 (h = lane & 31) of slice A, lanes 32-63 the
// same rows of slice B.  A value-code slice streams few matrix bytes, so its
// time goes to the vector accesses; with two rows per lane the codes, the
// column blocks, x (implicit columns), b, d and y all move in 16-B accesses
// (8-B-per-lane accesses run at ~0.5-0.7x the 16-B rate on MI355X).  Each row
// is still summed by one lane in ascending steps: bitwise unchanged.
typedef double dbl2u_t __attribute__((ext_vector_type(2), aligned(8)));

template <int MODE, int CM, int VB, int R>
__device__ __forceinline__ void sellc_group_rp(const char *__restrict__ blk, const char *__restrict__ ixb, int g,
                                               const int32_t *__restrict__ sa, const int32_t *__restrict__ sb,
                                               bool hb, int r0, const double *tab, const Epi &e, double &acc0,
                                               double &acc1) {
    const int t0 = 8 * g;
    uint32_t q0[4], q1[4];
    if constexpr (VB == 4) {
        const i32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x2_t *>(blk) + ((int64_t)g * SELL_C + r0) / 2);
        q0[0] = (uint32_t)v.x;
        q1[0] = (uint32_t)v.y;
    } else if constexpr (VB == 8) {
        const i32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t *>(blk) + ((int64_t)g * SELL_C + r0) / 2);
        q0[0] = (uint32_t)v.x;
        q0[1] = (uint32_t)v.y;
        q1[0] = (uint32_t)v.z;
        q1[1] = (uint32_t)v.w;
    } else {
        const i32x4_t *p = reinterpret_cast<const i32x4_t *>(blk) + (int64_t)g * SELL_C + r0;
        const i32x4_t v0 = __builtin_nontemporal_load(p);
        const i32x4_t v1 = __builtin_nontemporal_load(p + 1);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            q0[k] = (uint32_t)v0[k];
            q1[k] = (uint32_t)v1[k];
        }
    }
    int32_t bse[R];
#pragma unroll
    for (int u = 0; u < R; u++) bse[u] = hb ? sb[t0 + u] : sa[t0 + u];
    int32_t c0[R], c1[R];
    if constexpr (CM == 0) {
#pragma unroll
        for (int u = 0; u < R; u++) {
            c0[u] = bse[u] + r0;
            c1[u] = c0[u] + 1;
        }
    } else if constexpr (R == 8) {
        const int64_t el = (int64_t)t0 * SELL_C + 8 * r0;  // row r0: 8 elements, then row r0 + 1
        if constexpr (CM == 1) {
            const i32x4_t *p = reinterpret_cast<const i32x4_t *>(ixb + 2 * el);
            const i32x4_t d0 = __builtin_nontemporal_load(p);
            const i32x4_t d1 = __builtin_nontemporal_load(p + 1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                c0[2 * u] = bse[2 * u] + (int32_t)((uint32_t)d0[u] & 0xffffu);
                c0[2 * u + 1] = bse[2 * u + 1] + (int32_t)((uint32_t)d0[u] >> 16);
                c1[2 * u] = bse[2 * u] + (int32_t)((uint32_t)d1[u] & 0xffffu);
                c1[2 * u + 1] = bse[2 * u + 1] + (int32_t)((uint32_t)d1[u] >> 16);
            }
        } else {
            const i32x4_t *p = reinterpret_cast<const i32x4_t *>(ixb + 4 * el);
            const i32x4_t d0 = __builtin_nontemporal_load(p), d1 = __builtin_nontemporal_load(p + 1);
            const i32x4_t d2 = __builtin_nontemporal_load(p + 2), d3 = __builtin_nontemporal_load(p + 3);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                c0[u] = d0[u];
                c0[4 + u] = d1[u];
                c1[u] = d2[u];
                c1[4 + u] = d3[u];
            }
        }
    } else if constexpr (CM == 1) {
        // the 2R u16 of rows r0, r0 + 1 as R dwords (4-B aligned: r0 is even)
        // instead of 2R 2-B loads (P_0: 4-5 steps per row)
        const int64_t el = (int64_t)t0 * SELL_C + R * r0;
        const uint32_t *p = reinterpret_cast<const uint32_t *>(ixb + 2 * el);
        uint32_t dw[R];
#pragma unroll
        for (int k = 0; k < R; k++) dw[k] = __builtin_nontemporal_load(p + k);
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int j0 = u, j1 = R + u;  // element indices of the two rows
            c0[u] = bse[u] + (int32_t)((dw[j0 >> 1] >> (16 * (j0 & 1))) & 0xffffu);
            c1[u] = bse[u] + (int32_t)((dw[j1 >> 1] >> (16 * (j1 & 1))) & 0xffffu);
        }
    } else {
        const int64_t el = (int64_t)t0 * SELL_C + R * r0;  // row r0: R elements, then row r0 + 1
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int32_t *p = reinterpret_cast<const int32_t *>(ixb) + el;
            c0[u] = __builtin_nontemporal_load(p + u);
            c1[u] = __builtin_nontemporal_load(p + R + u);
        }
    }
    double x0[R], x1[R];
#pragma unroll
    for (int u = 0; u < R; u++) {
        if constexpr (CM == 0) {
            const dbl2_t v = *reinterpret_cast<const dbl2u_t *>(e.x + c0[u]);
            x0[u] = v.x;
            x1[u] = v.y;
        } else {
            x0[u] = e.x[c0[u]];
            x1[u] = e.x[c1[u]];
        }
    }
#pragma unroll
    for (int u = 0; u < R; u++) acc0 = fma(tab[sell_code<VB>(q0, u)], x0[u], acc0);
#pragma unroll
    for (int u = 0; u < R; u++) acc1 = fma(tab[sell_code<VB>(q1, u)], x1[u], acc1);
}

template <int MODE, int CM, int VB>
__device__ __forceinline__ void sellc_walk_rp(const char *ba, const char *bb, const int32_t *sa, const int32_t *sb,
                                              int w, int lane, const double *tab, const Epi &e, double &acc0,
                                              double &acc1) {
    const bool hb = lane >= 32;
    const int r0 = 2 * (lane & 31);
    const char *blk = hb ? bb : ba;
    const int ng = (w + 7) >> 3;
    const char *ixb = blk + (int64_t)ng * SELL_C * sell_code_bytes(VB);
    acc0 = 0.0;
    acc1 = 0.0;
    const int full = w >> 3;
    for (int g = 0; g < full; g++) sellc_group_rp<MODE, CM, VB, 8>(blk, ixb, g, sa, sb, hb, r0, tab, e, acc0, acc1);
    switch (w & 7) {
    case 1: sellc_group_rp<MODE, CM, VB, 1>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 2: sellc_group_rp<MODE, CM, VB, 2>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 3: sellc_group_rp<MODE, CM, VB, 3>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 4: sellc_group_rp<MODE, CM, VB, 4>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 5: sellc_group_rp<MODE, CM, VB, 5>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 6: sellc_group_rp<MODE, CM, VB, 6>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    case 7: sellc_group_rp<MODE, CM, VB, 7>(blk, ixb, full, sa, sb, hb, r0, tab, e, acc0, acc1); break;
    default: break;
    }
}

// Epilogue of two adjacent rows (row, row + 1) with 16-B accesses when both live.
// NT: b, d and y (streamed once, never gathered) bypass the caches.
template <int MODE, bool NT = false> struct EpiOps2 {
    dbl2_t xr = {0.0, 0.0}, br = {0.0, 0.0}, dr = {0.0, 0.0}, yr = {0.0, 0.0};
    int i = 0;
    bool l0 = false, l1 = false;
    __device__ __forceinline__ dbl2_t ld(const double *p) const {
        if (l1) return *reinterpret_cast<const dbl2u_t *>(p + i);
        dbl2_t v = {p[i], 0.0};
        return v;
    }
    __device__ __forceinline__ dbl2_t lds(const double *p) const {  // streamed operand
        if constexpr (NT) {
            if (l1) return __builtin_nontemporal_load(reinterpret_cast<const dbl2u_t *>(p + i));
            dbl2_t v = {__builtin_nontemporal_load(p + i), 0.0};
            return v;
        } else {
            return ld(p);
        }
    }
    __device__ __forceinline__ void load(const Epi &a, int row, bool live0, bool live1) {
        i = row;
        l0 = live0;
        l1 = live1;
        if (!l0) return;
        if constexpr (MODE == SPMV_JACOBI) {
            xr = ld(a.x);
            br = lds(a.b);
            if (a.dc) {
                dr.x = a.dt[a.dc[i]];
                dr.y = l1 ? a.dt[a.dc[i + 1]] : 0.0;
            } else {
                dr = lds(a.d);
            }
        }
        if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) br = lds(a.b);
        if constexpr (MODE == SPMV_ADD) yr = lds(a.y);
        if constexpr (MODE == SPMV_ADD0) {
            if (a.dc) {  // coded diagonal: 1 B per row instead of 8
                dr.x = a.dt[a.dc[i]];
                dr.y = l1 ? a.dt[a.dc[i + 1]] : 0.0;
                yr = dr * lds(a.b);
            } else {
                yr = lds(a.d) * lds(a.b);
            }
        }
    }
    __device__ __forceinline__ void store(const Epi &a, double acc0, double acc1) const {
        if (!l0) return;
        const dbl2_t acc = {acc0, acc1};
        dbl2_t out;
        if constexpr (MODE == SPMV_SET) out = acc;
        else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) out = yr + acc;
        else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) out = br - acc;
        else out = xr + dr * (br - acc);  // JACOBI
        if constexpr (NT) {
            if (l1) __builtin_nontemporal_store(out, reinterpret_cast<dbl2u_t *>(a.y + i));
            else __builtin_nontemporal_store(out.x, a.y + i);
        } else {
            if (l1) *reinterpret_cast<dbl2u_t *>(a.y + i) = out;
            else a.y[i] = out.x;
        }
    }
};

template <int MODE>
__host__ __device__ constexpr bool sell_row_pairs(int lay) {
    return lay >= 4 && (MODE == SPMV_SET || MODE == SPMV_ADD || MODE == SPMV_RESID || MODE == SPMV_JACOBI ||
                        MODE == SPMV_ADD0);
}

template <int MODE, int CM, int LAY>
__device__ __forceinline__ double sellc_walk_any(const char *blkp, const int32_t *bs, int w, int lane,
                                                 const double *stab, const SellArgs &a) {
    if constexpr (LAY == 16) return sellc_walk<MODE, CM, 16>(blkp, bs, w, lane, a.vtab, a.e);
    else return sellc_walk<MODE, CM, LAY>(blkp, bs, w, lane, stab, a.e);
}

// Slices per wave: one for fp64 values, two (in lockstep when their width and
// column mode agree) for value codes -- except RESID0, whose rows gather two
// vectors (d and x) and which ran slower with the doubled register footprint.
__host__ __device__ constexpr int sell_slices_per_wave(int lay, int mode) {
    return lay >= 4 && mode != SPMV_RESID0 ? 2 : 1;
}

// LAY: 0 one step per 512-B row, 1 step pairs (fp64 values); 4 / 8 / 16 value codes
template <int MODE, int LAY>
__device__ __forceinline__ void sell_wave(const SellArgs &a, const double *stab, int sl) {
    const int slice = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    if constexpr (sell_row_pairs<MODE>(LAY) && sell_slices_per_wave(LAY, MODE) == 2) {
        // two slices of equal width and column mode: two adjacent rows per lane
        if (a.spw == 2 && sl + 1 < a.nslices) {
            const int ta = a.soff[slice], tb = a.soff[slice + 1], te = a.soff[slice + 2];
            const uint32_t da = a.desc[slice], db = a.desc[slice + 1];
            if (tb - ta == te - tb && (da >> 30) == (db >> 30)) {
                const bool hb = lane >= 32;
                const int rs = hb ? a.row0[slice + 1] : a.row0[slice];
                const int re = hb ? a.row0[slice + 2] : a.row0[slice + 1];
                const int row = rs + 2 * (lane & 31);
                EpiOps2<MODE> ep2;
                ep2.load(a.e, row, row < re, row + 1 < re);
                const char *ba = a.data + (int64_t)(da & 0x3fffffffu) * 128;
                const char *bb = a.data + (int64_t)(db & 0x3fffffffu) * 128;
                const int32_t *sa = a.base + ta, *sbp = a.base + tb;
                const double *tab = LAY == 16 ? a.vtab : stab;
                double acc0, acc1;
                switch (da >> 30) {
                case 0: sellc_walk_rp<MODE, 0, LAY>(ba, bb, sa, sbp, tb - ta, lane, tab, a.e, acc0, acc1); break;
                case 1: sellc_walk_rp<MODE, 1, LAY>(ba, bb, sa, sbp, tb - ta, lane, tab, a.e, acc0, acc1); break;
                default: sellc_walk_rp<MODE, 2, LAY>(ba, bb, sa, sbp, tb - ta, lane, tab, a.e, acc0, acc1); break;
                }
                ep2.store(a.e, acc0, acc1);
                return;
            }
        }
    }
    const int row = a.row0[slice] + lane;
    const bool live = row < a.row0[slice + 1];
    EpiOps<MODE> ep;
    if (live) ep.load(a.e, row);
    const int t0 = a.soff[slice];
    const int w = a.soff[slice + 1] - t0;
    const uint32_t d = a.desc[slice];
    const char *blkp = a.data + (int64_t)(d & 0x3fffffffu) * 128;
    const int32_t *bs = a.base + t0;
    double acc;
    if (LAY >= 4 && (sell_slices_per_wave(LAY, MODE) == 1 || a.spw == 1)) {
        switch (d >> 30) {
        case 0: acc = sellc_walk_any<MODE, 0, LAY>(blkp, bs, w, lane, stab, a); break;
        case 1: acc = sellc_walk_any<MODE, 1, LAY>(blkp, bs, w, lane, stab, a); break;
        default: acc = sellc_walk_any<MODE, 2, LAY>(blkp, bs, w, lane, stab, a); break;
        }
    } else if constexpr (LAY >= 4) {
        // second slice of the wave
        const bool two = sl + 1 < a.nslices;
        int rowb = 0, wb = 0;
        bool liveb = false;
        uint32_t db = 0;
        EpiOps<MODE> epb;
        if (two) {
            rowb = a.row0[slice + 1] + lane;
            liveb = rowb < a.row0[slice + 2];
            if (liveb) epb.load(a.e, rowb);
            wb = a.soff[slice + 2] - a.soff[slice + 1];
            db = a.desc[slice + 1];
        }
        const char *blkb = a.data + (int64_t)(db & 0x3fffffffu) * 128;
        const int32_t *bsb = a.base + t0 + w;
        double accb = 0.0;
        if (two && wb == w && (db >> 30) == (d >> 30)) {
            switch (d >> 30) {
            case 0: sellc_walk2<MODE, 0, LAY>(blkp, blkb, bs, bsb, w, lane, LAY == 16 ? a.vtab : stab, a.e, acc, accb); break;
            case 1: sellc_walk2<MODE, 1, LAY>(blkp, blkb, bs, bsb, w, lane, LAY == 16 ? a.vtab : stab, a.e, acc, accb); break;
            default: sellc_walk2<MODE, 2, LAY>(blkp, blkb, bs, bsb, w, lane, LAY == 16 ? a.vtab : stab, a.e, acc, accb); break;
            }
        } else {
            switch (d >> 30) {
            case 0: acc = sellc_walk_any<MODE, 0, LAY>(blkp, bs, w, lane, stab, a); break;
            case 1: acc = sellc_walk_any<MODE, 1, LAY>(blkp, bs, w, lane, stab, a); break;
            default: acc = sellc_walk_any<MODE, 2, LAY>(blkp, bs, w, lane, stab, a); break;
            }
            if (two) {
                switch (db >> 30) {
                case 0: accb = sellc_walk_any<MODE, 0, LAY>(blkb, bsb, wb, lane, stab, a); break;
                case 1: accb = sellc_walk_any<MODE, 1, LAY>(blkb, bsb, wb, lane, stab, a); break;
                default: accb = sellc_walk_any<MODE, 2, LAY>(blkb, bsb, wb, lane, stab, a); break;
                }
            }
        }
        if (live) ep.store(a.e, acc);
        if (liveb) epb.store(a.e, accb);
        return;
    } else if constexpr (LAY == 1) {
        switch (d >> 30) {
        case 0: acc = sell_walk_pairs<MODE, 0>(blkp, bs, w, lane, a.e); break;
        case 1: acc = sell_walk_pairs<MODE, 1>(blkp, bs, w, lane, a.e); break;
        default: acc = sell_walk_pairs<MODE, 2>(blkp, bs, w, lane, a.e); break;
        }
    } else {
        switch (d >> 30) {
        case 0: acc = sell_walk_steps<MODE, 0>(blkp, bs, w, lane, a.e); break;
        case 1: acc = sell_walk_steps<MODE, 1>(blkp, bs, w, lane, a.e); break;
        default: acc = sell_walk_steps<MODE, 2>(blkp, bs, w, lane, a.e); break;
        }
    }
    if (live) ep.store(a.e, acc);
}


// Consecutive slice groups per wave (1: four per wave made the small coarse
// levels launch too few waves and did not speed up the fine level).
__host__ __device__ constexpr int sell_groups_per_wave(int) { return 1; }

template <int MODE, int LAY>
__global__ __launch_bounds__(256) void spmv_sell_kernel(SellArgs a) {
    constexpr int TABN = LAY == 4 ? 16 : LAY == 8 ? 256 : 1;
    __shared__ double stab[TABN];
    if constexpr (LAY == 4 || LAY == 8) {
        for (int i = threadIdx.x; i < a.ntab; i += 256) stab[i] = a.vtab[i];
        __syncthreads();
    }
    constexpr int SPW = sell_slices_per_wave(LAY, MODE);
    constexpr int NSEQ = sell_groups_per_wave(LAY);
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int wv = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    for (int k = 0; k < NSEQ; k++) {
        const int sl = (wv * NSEQ + k) * (SPW == 2 ? a.spw : 1);
        if (sl >= a.nslices) return;
        sell_wave<MODE, LAY>(a, stab, sl);
    }
}

// 16-bit codes with the table staged in LDS (dynamic, ntab doubles) by a
// persistent grid: each workgroup stages once and walks virtual blocks v, v + G,
// ... of the spmv_sell_kernel decomposition (the table reads become LDS reads
// instead of dependent L2 gathers; per-block staging alone measured slower).
template <int MODE>
__global__ __launch_bounds__(256) void spmv_sell_t16_kernel(SellArgs a, int nvb) {
    extern __shared__ double dtab[];
    for (int i = threadIdx.x; i < a.ntab; i += 256) dtab[i] = a.vtab[i];
    __syncthreads();
    SellArgs b = a;
    b.vtab = dtab;
    constexpr int SPW = sell_slices_per_wave(16, MODE);
    for (int v = blockIdx.x; v < nvb; v += gridDim.x) {
        const int blk = xcd_remap(v, nvb);
        const int wv = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
        const int sl = wv * (SPW == 2 ? b.spw : 1);
        if (sl < b.nslices) sell_wave<MODE, 16>(b, nullptr, sl);
    }
}

// 16-bit-code SELL with its table in LDS for long rows (>= 32 entries on average:
// R_1 of the 256^3 cycle, 87 entries per row, 40 -> 35 us; short rows such as P_1's
// 11 pay more for the staging than they save: 47 -> 48 us with a persistent grid
// of 2 workgroups per CU, 56 us with 4).  A/B switch FAMG_SELL_T16=0: off; N > 0:
// also for short rows, at most N workgroups per CU.
static int sell_t16_mode() {
    static const int v = [] {
        const char *e = getenv("FAMG_SELL_T16");
        return e ? atoi(e) : -1;
    }();
    return v;
}

// Value-code SELL whose slices are all at most 4 steps wide with implicit or
// u16 columns and pair up (equal width and column mode): P_0 of a box
// hierarchy (4 entries per row).  Only the lockstep row-pair path of
// spmv_sell_kernel, with R = w known per case: a fraction of the generic
// kernel's registers (which it sizes for 8-step groups of every layout), so
// more waves keep their loads in flight.  Same row sums in the same order.
template <int MODE, int LAY>
__global__ __launch_bounds__(256) void spmv_sell_short_kernel(SellArgs a) {
    constexpr int TABN = LAY == 4 ? 16 : LAY == 8 ? 256 : 1;
    __shared__ double stab[TABN];
    if constexpr (LAY == 4 || LAY == 8) {
        for (int i = threadIdx.x; i < a.ntab; i += 256) stab[i] = a.vtab[i];
        __syncthreads();
    }
    const double *tab = LAY == 16 ? a.vtab : stab;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = 2 * __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int slice = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int ta = a.soff[slice], tb = a.soff[slice + 1];
    const uint32_t da = a.desc[slice], db = a.desc[slice + 1];
    const bool hb = lane >= 32;
    const int rs = hb ? a.row0[slice + 1] : a.row0[slice];
    const int re = hb ? a.row0[slice + 2] : a.row0[slice + 1];
    const int row = rs + 2 * (lane & 31);
    // ADD0 (the folded correction d*b + P x): its operands are loaded here and the
    // coded diagonal decoded after the row's loads are issued (EpiOps2 decodes it
    // first, and the dependent table read held up the row: 119 vs 99 us for ADD)
    constexpr bool A0 = MODE == SPMV_ADD0;
    EpiOps2<A0 ? SPMV_SET : MODE> ep2;
    const bool l0 = row < re, l1 = row + 1 < re;
    ep2.load(a.e, row, l0, l1);
    dbl2_t b0 = {0.0, 0.0}, d0 = {0.0, 0.0};
    uint32_t k0 = 0, k1 = 0;
    if constexpr (A0) {
        if (l0) {
            if (l1) b0 = *reinterpret_cast<const dbl2u_t *>(a.e.b + row);
            else b0.x = a.e.b[row];
            if (a.e.dc) {
                k0 = a.e.dc[row];
                k1 = a.e.dc[l1 ? row + 1 : row];
            } else if (l1) {
                d0 = *reinterpret_cast<const dbl2u_t *>(a.e.d + row);
            } else {
                d0.x = a.e.d[row];
            }
        }
    }
    const char *blk2 = a.data + (int64_t)((hb ? db : da) & 0x3fffffffu) * 128;
    const char *ixb = blk2 + (int64_t)SELL_C * sell_code_bytes(LAY);
    const int32_t *sa = a.base + ta, *sbp = a.base + tb;
    const int r0 = 2 * (lane & 31);
    double acc0 = 0.0, acc1 = 0.0;
    switch ((int)(da >> 30) * 8 + (tb - ta)) {
    case 1: sellc_group_rp<MODE, 0, LAY, 1>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 2: sellc_group_rp<MODE, 0, LAY, 2>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 3: sellc_group_rp<MODE, 0, LAY, 3>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 4: sellc_group_rp<MODE, 0, LAY, 4>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 9: sellc_group_rp<MODE, 1, LAY, 1>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 10: sellc_group_rp<MODE, 1, LAY, 2>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 11: sellc_group_rp<MODE, 1, LAY, 3>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    case 12: sellc_group_rp<MODE, 1, LAY, 4>(blk2, ixb, 0, sa, sbp, hb, r0, tab, a.e, acc0, acc1); break;
    default: break;  // width 0
    }
    if constexpr (A0) {
        if (!l0) return;
        if (a.e.dc) {
            d0.x = a.e.dt[k0];
            d0.y = l1 ? a.e.dt[k1] : 0.0;
        }
        const dbl2_t out = d0 * b0 + dbl2_t{acc0, acc1};
        if (l1) *reinterpret_cast<dbl2u_t *>(a.e.y + row) = out;
        else a.e.y[row] = out.x;
    } else {
        ep2.store(a.e, acc0, acc1);
    }
}

// ---------------------------------------------------------------- DIA codes
//
// A square matrix whose entries lie on at most DIA_MAX diagonals (the union of
// col - row offsets; a constant stencil: 7 for the 7-pt Laplacian, 27 for the
// 27-pt operator), that fills them to >= 80 % and whose values have a 4/8-bit
// value table is stored as one code word group per row: the codes of its K
// diagonals, ascending offset (= ascending column, the stored order), with
// the +0.0 code where a row has no entry.  No per-slice metadata exists, so a
// row's only dependent chain is code + x loads -> fma -> store; each lane takes
// two adjacent rows (16-B accesses throughout).  x indices outside [0, ncols)
// belong to padding entries (value 0.0) and are clamped.
constexpr int DIA_MAX = 40;  // 32 for the generic kernels; longer stencils through a run pattern

struct DiaArgs {
    const uint32_t *codes;  // cw words per row (rows padded by 2)
    const double *vtab;
    int32_t ntab, k, row_begin, row_end, ncols;
    int32_t code_row0;  // first row with codes (the DIA row range may be one segment)
    int32_t band_bp;    // > 0: 512-row blocks per plane; XCD x walks band x of every plane
    int32_t off[DIA_MAX];
    Epi e;
    int32_t gnx, gny, gnz;  // CST: the grid (nx even)
    double cst[27];         // CST: the interior stencil
};

typedef int32_t i32x2u_t __attribute__((ext_vector_type(2), aligned(4)));
typedef int32_t i32x4u_t __attribute__((ext_vector_type(4), aligned(4)));

// x operands of rows (r, r+1) at column c = r + off: x[clamp(c)], x[clamp(c+1)]
// from one 16-B load at clamp(c, 0, ncols-2) and selects -- branch-free, so
// the loads of all diagonals stay in flight together (a divergent edge path
// made the compiler wait for each load at its join).  Needs ncols >= 2.
template <int MODE> __device__ __forceinline__ void dia_gx2(const Epi &e, int c, int ncols, double &x0, double &x1) {
    const int cc = min(max(c, 0), ncols - 2);
    dbl2_t v = *reinterpret_cast<const dbl2u_t *>(e.x + cc);
    if constexpr (MODE == SPMV_RESID0) v = *reinterpret_cast<const dbl2u_t *>(e.d + cc) * v;
    x0 = c > ncols - 2 ? v.y : v.x;
    x1 = c < 0 ? v.x : v.y;
}

template <int CW>
__device__ __forceinline__ void dia_codes2(const uint32_t *cp, uint32_t (&w0)[CW], uint32_t (&w1)[CW]) {
    if constexpr (CW == 1) {
        const i32x2u_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x2u_t *>(cp));
        w0[0] = (uint32_t)v.x;
        w1[0] = (uint32_t)v.y;
    } else if constexpr (CW == 2) {
        const i32x4u_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4u_t *>(cp));
        w0[0] = (uint32_t)v.x;
        w0[1] = (uint32_t)v.y;
        w1[0] = (uint32_t)v.z;
        w1[1] = (uint32_t)v.w;
    } else {
#pragma unroll
        for (int q = 0; q < CW / 4; q++) {
            const i32x4u_t v0 = __builtin_nontemporal_load(reinterpret_cast<const i32x4u_t *>(cp) + q);
            const i32x4u_t v1 = __builtin_nontemporal_load(reinterpret_cast<const i32x4u_t *>(cp + CW) + q);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                w0[4 * q + j] = (uint32_t)v0[j];
                w1[4 * q + j] = (uint32_t)v1[j];
            }
        }
    }
}

// The weighted-Jacobi epilogue with the 8-bit coded diagonal (d = dt[dc[i]],
// dt padded to 256 entries and staged in LDS with the value table).
constexpr int DIA_JACOBI_DC = 16;
// The folded zero-guess residual y = b - A (d x) with the 8-bit coded diagonal:
// the 7-point kernel gathers the 1-B codes of d beside x (dt staged in LDS)
// instead of 8-B values of d: 17 MB instead of 134 MB more than a residual.
constexpr int DIA_RESID0_DC = 17;
// The same two epilogues when the coded diagonal is one value (Epi::dk: the 7-point
// Laplacian's a_ii = 6 everywhere): d is one scalar load, no per-row or gathered
// codes (the 7-point run kernel only)
constexpr int DIA_JACOBI_DK = 18;
constexpr int DIA_RESID0_DK = 19;

// 8-bit codes at the positions dia_gx2 / dia_gx4 take their x operands from
// (same clamps and selects)
__device__ __forceinline__ void dia_gc2(const uint8_t *dc, int c, int ncols, uint32_t &k0, uint32_t &k1) {
    const int cc = min(max(c, 0), ncols - 2);
    const uint32_t a0 = dc[cc], a1 = dc[cc + 1];
    k0 = c > ncols - 2 ? a1 : a0;
    k1 = c < 0 ? a0 : a1;
}
__device__ __forceinline__ void dia_gc4(const uint8_t *dc, int c, int ncols, uint32_t (&k)[4]) {
    const int p0 = min(max(c, 0), ncols - 2), p1 = min(max(c + 2, 0), ncols - 2);
    const uint32_t a0 = dc[p0], a1 = dc[p0 + 1], b0 = dc[p1], b1 = dc[p1 + 1];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int t = c + j;
        k[j] = t == p0 ? a0 : t == p0 + 1 ? a1 : t == p1 ? b0 : b1;
    }
}

// Epilogue operands of a DIA row pair, loaded without divergence: one 16-B
// load at i2 = min(row, row_end - 2) per vector; a tail row (row_end - 1)
// takes the upper half.  Lanes past row_end load in-range data and store
// nothing.
template <int MODE, bool NT> struct DiaEpi {
    dbl2_t xr = {0.0, 0.0}, br = {0.0, 0.0}, dr = {0.0, 0.0}, yr = {0.0, 0.0};
    int row = 0, i2 = 0;
    uint32_t dc0 = 0, dc1 = 0;
    bool l0 = false, l1 = false;
    __device__ __forceinline__ dbl2_t ldv(const double *p) const {
        const dbl2u_t *q = reinterpret_cast<const dbl2u_t *>(p + i2);
        dbl2_t v = NT ? __builtin_nontemporal_load(q) : *q;
        if (row != i2) v.x = v.y;
        return v;
    }
    // the diagonal codes are loaded first: waiting for them later waits for nothing else
    __device__ __forceinline__ void load_codes(const Epi &a, int r, int row_end) {
        if constexpr (MODE == DIA_JACOBI_DC) {
            dc0 = a.dc[min(r, row_end - 1)];
            dc1 = a.dc[min(r + 1, row_end - 1)];
        }
    }
    __device__ __forceinline__ void load(const Epi &a, int r, int row_end) {
        row = r;
        i2 = min(r, row_end - 2);
        l0 = r < row_end;
        l1 = r + 1 < row_end;
        if constexpr (MODE == SPMV_JACOBI || MODE == DIA_JACOBI_DC || MODE == DIA_JACOBI_DK) {
            const dbl2u_t *q = reinterpret_cast<const dbl2u_t *>(a.x + i2);  // x is gathered: cached
            xr = *q;
            if (row != i2) xr.x = xr.y;
            br = ldv(a.b);
        }
        if constexpr (MODE == SPMV_JACOBI) dr = ldv(a.d);
        if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0 || MODE == DIA_RESID0_DC || MODE == DIA_RESID0_DK)
            br = ldv(a.b);
        if constexpr (MODE == SPMV_ADD) yr = ldv(a.y);
        if constexpr (MODE == SPMV_ADD0) yr = ldv(a.d) * ldv(a.b);
    }
    __device__ __forceinline__ void store(const Epi &a, const double *sdt, double acc0, double acc1) {
        const dbl2_t acc = {acc0, acc1};
        dbl2_t out;
        if constexpr (MODE == DIA_JACOBI_DC) dr = dbl2_t{sdt[dc0], sdt[dc1]};
        if constexpr (MODE == SPMV_SET) out = acc;
        else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) out = yr + acc;
        else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0 || MODE == DIA_RESID0_DC || MODE == DIA_RESID0_DK)
            out = br - acc;
        else out = xr + dr * (br - acc);  // JACOBI
        if (l1) {
            if constexpr (NT) __builtin_nontemporal_store(out, reinterpret_cast<dbl2u_t *>(a.y + row));
            else *reinterpret_cast<dbl2u_t *>(a.y + row) = out;
        } else if (l0) {
            if constexpr (NT) __builtin_nontemporal_store(out.x, a.y + row);
            else a.y[row] = out.x;
        }
    }
};

// Two adjacent rows per lane, 512 rows per workgroup.  Every load is issued
// unconditionally (clamped indices; all KMAX diagonals, off[k] = 0 past K,
// whose terms are not added), so no load waits on another -- a divergent edge
// path or a per-diagonal guard made the compiler wait for each load at the
// join.  The value table (and the coded diagonal's table) is fetched first and
// published to LDS behind an LDS-only barrier after the row loads are issued,
// so they stay in flight across it.
// x[c .. c+3] of rows (r, r+1) for a run of three diagonals (offsets o-1, o, o+1,
// c = r + o - 1) from two 16-B loads at clamp(c) and clamp(c + 2); selects keep
// every in-range position exact at the matrix edges (out-of-range positions
// belong to +0.0 terms).
template <int MODE>
__device__ __forceinline__ void dia_gx4(const Epi &e, int c, int ncols, double (&v)[4]) {
    const int p0 = min(max(c, 0), ncols - 2), p1 = min(max(c + 2, 0), ncols - 2);
    dbl2_t q0 = *reinterpret_cast<const dbl2u_t *>(e.x + p0);
    dbl2_t q1 = *reinterpret_cast<const dbl2u_t *>(e.x + p1);
    if constexpr (MODE == SPMV_RESID0) {
        q0 = *reinterpret_cast<const dbl2u_t *>(e.d + p0) * q0;
        q1 = *reinterpret_cast<const dbl2u_t *>(e.d + p1) * q1;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int t = c + j;
        v[j] = t == p0 ? q0.x : t == p0 + 1 ? q0.y : t == p1 ? q1.x : q1.y;
    }
}

// NR > 0: the K = 3 NR diagonals come in runs of three consecutive offsets (a
// 27-point stencil: NR = 9); a row pair's three x operands per run are four
// consecutive values, two 16-B loads instead of three and 4 NR instead of 2 KMAX
// registers.  NR = -1: the 7-point pattern (single, single, run of three,
// single, single).  The row sums run over the same diagonals in the same order.
// CST (7-point run kernel, dia_constant): no codes, the interior coefficients
// from the arguments, x operands of neighbours outside the grid taken as 0.0
// (bitwise the coded sums, as spmv_dia_pat_kernel CST)
template <int MODE, int VB, int CW, bool NT, int NR = 0, bool CST = false>
__global__ __launch_bounds__(256) void spmv_dia_kernel(DiaArgs a) {
    constexpr bool DC = MODE == DIA_JACOBI_DC;
    constexpr bool RC = MODE == DIA_RESID0_DC && NR == -1;  // coded d gathered beside x
    constexpr bool JK = MODE == DIA_JACOBI_DK, RK = MODE == DIA_RESID0_DK;  // d = dt[0]
    static_assert(!(JK || RK) || NR == -1, "constant-d epilogues: 7-point run kernel only");
    // x operand of the row sums (RC, RK: plain x, multiplied by d after the loads)
    constexpr int GM = DC || JK ? SPMV_JACOBI : RC || RK ? SPMV_SET : MODE == DIA_RESID0_DC ? SPMV_RESID0 : MODE;
    double dk = 0.0;
    if constexpr (JK || RK) dk = a.e.dk;
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[DC || RC ? 256 : 1];
    const double tv = (int)threadIdx.x < a.ntab ? a.vtab[threadIdx.x] : 0.0;
    double dv = 0.0;
    if constexpr (DC || RC) dv = a.e.dt[threadIdx.x];
    int blk;
    if (a.band_bp > 0) {
        // 2.5-D order: XCD x takes band x (1/8 of the rows) of every plane in
        // turn, so its x window is three plane bands (768 KB at 512^2 planes),
        // not three whole planes (6 MB > its 4 MB L2)
        const int bb = a.band_bp >> 3, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        blk = (i / bb) * a.band_bp + x * bb + (i % bb);
    } else {
        blk = xcd_remap(blockIdx.x, gridDim.x);
    }
    const int row = a.row_begin + 512 * blk + 2 * (int)threadIdx.x;
    constexpr int KMAX = CW * 32 / VB < DIA_MAX ? CW * 32 / VB : DIA_MAX;
    constexpr uint32_t MASK = (1u << VB) - 1;
    constexpr int KX = NR != 0 ? 1 : KMAX;  // per-diagonal operands (generic path)
    constexpr int NRX = NR > 0 ? NR : 1;    // per-run operands (run path)
    DiaEpi<MODE, NT> ep;
    uint32_t w0[CW], w1[CW];
    double x0[KX], x1[KX], xq[NRX][4];
    ep.load_codes(a.e, row, a.row_end);
    ep.load(a.e, row, a.row_end);
    static_assert(!CST || NR == -1, "constant stencils: the 7-point run kernel");
    if constexpr (!CST) dia_codes2<CW>(a.codes + (int64_t)(min(row, a.row_end - 1) - a.code_row0) * CW, w0, w1);
    double xs7[4][2];  // NR == -1 (7-point): the four single diagonals
    uint32_t ks7[4][2], kq[4];  // RC: their codes of d
    if constexpr (RC) {
        dia_gc2(a.e.dc, row + a.off[0], a.ncols, ks7[0][0], ks7[0][1]);
        dia_gc2(a.e.dc, row + a.off[1], a.ncols, ks7[1][0], ks7[1][1]);
        dia_gc4(a.e.dc, row + a.off[2], a.ncols, kq);
        dia_gc2(a.e.dc, row + a.off[5], a.ncols, ks7[2][0], ks7[2][1]);
        dia_gc2(a.e.dc, row + a.off[6], a.ncols, ks7[3][0], ks7[3][1]);
    }
    if constexpr (NR > 0) {
#pragma unroll
        for (int j = 0; j < NR; j++) dia_gx4<GM>(a.e, row + a.off[3 * j], a.ncols, xq[j]);
    } else if constexpr (NR == -1) {
        dia_gx2<GM>(a.e, row + a.off[0], a.ncols, xs7[0][0], xs7[0][1]);
        dia_gx2<GM>(a.e, row + a.off[1], a.ncols, xs7[1][0], xs7[1][1]);
        dia_gx4<GM>(a.e, row + a.off[2], a.ncols, xq[0]);
        dia_gx2<GM>(a.e, row + a.off[5], a.ncols, xs7[2][0], xs7[2][1]);
        dia_gx2<GM>(a.e, row + a.off[6], a.ncols, xs7[3][0], xs7[3][1]);
    } else {
#pragma unroll
        for (int k = 0; k < KMAX; k++) dia_gx2<GM>(a.e, row + a.off[k], a.ncols, x0[k], x1[k]);
    }
    if ((int)threadIdx.x < a.ntab) stab[threadIdx.x] = tv;
    if constexpr (DC || RC) sdt[threadIdx.x] = dv;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (row >= a.row_end) return;
    if constexpr (RC) {  // the zero-guess iterate d*x per column (vec_mul's product)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) xs7[i][j] = sdt[ks7[i][j]] * xs7[i][j];
#pragma unroll
        for (int j = 0; j < 4; j++) xq[0][j] = sdt[kq[j]] * xq[0][j];
    }
    if constexpr (RK) {  // the same product with the one value of d
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) xs7[i][j] = dk * xs7[i][j];
#pragma unroll
        for (int j = 0; j < 4; j++) xq[0][j] = dk * xq[0][j];
    }
    if constexpr (JK) ep.dr = dbl2_t{dk, dk};
    double acc0 = 0.0, acc1 = 0.0;
    if constexpr (NR == -1 && CST) {
        // diagonals z-1, y-1, x-1, 0, x+1, y+1, z+1; the row pair shares its grid row
        const int q = row / a.gnx, gx = row - q * a.gnx;
        const int gz = q / a.gny, gy = q - gz * a.gny;
        const bool zlo = gz > 0, ylo = gy > 0, yhi = gy < a.gny - 1, zhi = gz < a.gnz - 1;
        const bool xlo = gx > 0, xhi = gx + 2 < a.gnx;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double y0 = k < 2 ? xs7[k][0] : k < 5 ? xq[0][k - 2] : xs7[k - 3][0];
            const double y1 = k < 2 ? xs7[k][1] : k < 5 ? xq[0][k - 1] : xs7[k - 3][1];
            const bool in = k == 0 ? zlo : k == 1 ? ylo : k == 5 ? yhi : k == 6 ? zhi : true;
            const bool in0 = in && (k != 2 || xlo), in1 = in && (k != 4 || xhi);
            acc0 = fma(a.cst[k], in0 ? y0 : 0.0, acc0);
            acc1 = fma(a.cst[k], in1 ? y1 : 0.0, acc1);
        }
    } else if constexpr (NR == -1) {
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double y0 = k < 2 ? xs7[k][0] : k < 5 ? xq[0][k - 2] : xs7[k - 3][0];
            const double y1 = k < 2 ? xs7[k][1] : k < 5 ? xq[0][k - 1] : xs7[k - 3][1];
            acc0 = fma(stab[(w0[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], y0, acc0);
            acc1 = fma(stab[(w1[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], y1, acc1);
        }
    } else if constexpr (NR > 0) {
#pragma unroll
        for (int k = 0; k < 3 * NR; k++) {
            acc0 = fma(stab[(w0[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], xq[k / 3][k % 3], acc0);
            acc1 = fma(stab[(w1[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], xq[k / 3][k % 3 + 1], acc1);
        }
    } else {
#pragma unroll
        for (int k = 0; k < KMAX; k++) {
            const double f0 = fma(stab[(w0[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], x0[k], acc0);
            const double f1 = fma(stab[(w1[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], x1[k], acc1);
            acc0 = k < a.k ? f0 : acc0;
            acc1 = k < a.k ? f1 : acc1;
        }
    }
    ep.store(a.e, sdt, acc0, acc1);
}

// The constant 7-point kernel (CST above) with RP row pairs per lane (FLAG_DIA7_RP:
// 0 auto = 2 for SET, or 2 / 4): a workgroup covers RP adjacent 512-row blocks and issues every load
// of all its row pairs before the first sum -- RP times the bytes in flight per
// wave, fewer and longer-lived workgroups.  Same sums and epilogues, bitwise.
// (Coded-diagonal epilogues, which stage a table in LDS, stay on the kernel above.)
template <int MODE, int RP>
__global__ __launch_bounds__(256) void spmv_dia7c_kernel(DiaArgs a) {
    constexpr bool JK = MODE == DIA_JACOBI_DK, RK = MODE == DIA_RESID0_DK;
    constexpr int GM = JK ? SPMV_JACOBI : RK ? SPMV_SET : MODE;
    int blk;
    if (a.band_bp > 0) {  // the 2.5-D band order in units of RP blocks
        const int bp = a.band_bp / RP, bb = bp >> 3, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        blk = (i / bb) * bp + x * bb + (i % bb);
    } else {
        blk = xcd_remap(blockIdx.x, gridDim.x);
    }
    DiaEpi<MODE, false> ep[RP];
    double xs7[RP][4][2], xq[RP][4];
    int row[RP];
#pragma unroll
    for (int p = 0; p < RP; p++) {
        row[p] = a.row_begin + 512 * (RP * blk + p) + 2 * (int)threadIdx.x;
        ep[p].load(a.e, row[p], a.row_end);
        dia_gx2<GM>(a.e, row[p] + a.off[0], a.ncols, xs7[p][0][0], xs7[p][0][1]);
        dia_gx2<GM>(a.e, row[p] + a.off[1], a.ncols, xs7[p][1][0], xs7[p][1][1]);
        dia_gx4<GM>(a.e, row[p] + a.off[2], a.ncols, xq[p]);
        dia_gx2<GM>(a.e, row[p] + a.off[5], a.ncols, xs7[p][2][0], xs7[p][2][1]);
        dia_gx2<GM>(a.e, row[p] + a.off[6], a.ncols, xs7[p][3][0], xs7[p][3][1]);
    }
#pragma unroll
    for (int p = 0; p < RP; p++) {
        if (row[p] >= a.row_end) break;  // the row pairs ascend
        if constexpr (RK) {
            const double dk = a.e.dk;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) xs7[p][i][j] = dk * xs7[p][i][j];
#pragma unroll
            for (int j = 0; j < 4; j++) xq[p][j] = dk * xq[p][j];
        }
        if constexpr (JK) ep[p].dr = dbl2_t{a.e.dk, a.e.dk};
        const int q = row[p] / a.gnx, gx = row[p] - q * a.gnx;
        const int gz = q / a.gny, gy = q - gz * a.gny;
        const bool zlo = gz > 0, ylo = gy > 0, yhi = gy < a.gny - 1, zhi = gz < a.gnz - 1;
        const bool xlo = gx > 0, xhi = gx + 2 < a.gnx;
        double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double y0 = k < 2 ? xs7[p][k][0] : k < 5 ? xq[p][k - 2] : xs7[p][k - 3][0];
            const double y1 = k < 2 ? xs7[p][k][1] : k < 5 ? xq[p][k - 1] : xs7[p][k - 3][1];
            const bool in = k == 0 ? zlo : k == 1 ? ylo : k == 5 ? yhi : k == 6 ? zhi : true;
            const bool in0 = in && (k != 2 || xlo), in1 = in && (k != 4 || xhi);
            acc0 = fma(a.cst[k], in0 ? y0 : 0.0, acc0);
            acc1 = fma(a.cst[k], in1 ? y1 : 0.0, acc1);
        }
        ep[p].store(a.e, nullptr, acc0, acc1);
    }
}

// Run patterns of longer stencils (more than 32 diagonals): the lengths of the
// runs of consecutive offsets, ascending.  PAT 33: the Galerkin operator of
// smoothed aggregation on 2^3 boxes of the 7-point operator (A_1 of the C2
// cycle: the 27 neighbours in {-1,0,1}^3 plus +-2 along each axis) --
// z-2 | three x runs in z-1 | y-2 | x run | x run of five | x run | y+2 |
// three x runs in z+1 | z+2.
// PAT 27: the 27-point stencil, nine x runs of three.
__host__ __device__ constexpr int dia_pat_nrun(int pat) { return pat == 33 ? 13 : pat == 27 ? 9 : 0; }
__host__ __device__ constexpr int dia_pat_len(int pat, int j) {
    return pat == 33 ? (j == 0 || j == 4 || j == 8 || j == 12 ? 1 : j == 6 ? 5 : 3) : pat == 27 ? 3 : 0;
}
__host__ __device__ constexpr int dia_pat_k(int pat) {
    int s = 0;
    for (int j = 0; j < dia_pat_nrun(pat); j++) s += dia_pat_len(pat, j);
    return s;
}
// x registers of run j for a row pair: L + 1 values from (L + 2) / 2 16-B loads
__host__ __device__ constexpr int dia_pat_nq(int pat, int j) { return (dia_pat_len(pat, j) + 2) / 2; }
__host__ __device__ constexpr int dia_pat_nv(int pat) {
    int s = 0;
    for (int j = 0; j < dia_pat_nrun(pat); j++) s += 2 * dia_pat_nq(pat, j);
    return s;
}

// The DIA kernel for a run pattern: two rows per lane as spmv_dia_kernel; run
// j (L diagonals, first offset o) reads x[c .. c+L] of the row pair (c = row +
// o) with (L+2)/2 16-B loads at clamp(c + 2q); value c + i sits in load i/2
// (low half iff it is the load's clamped position), exact for every in-range
// column (out-of-range ones belong to +0.0 terms and read some finite x).
// Codes: cw words per row (not a power of two), the row pair's 2 cw words
// loaded as 16-B + 8-B + 4-B pieces.  Row sums over the K diagonals in
// ascending order, as the other DIA kernels.
template <int GM, int PAT, bool CLAMP>
__device__ __forceinline__ void dia_pat_loads(const DiaArgs &a, int row, double (&xv)[dia_pat_nv(PAT)]) {
    int kd = 0, vo = 0;
#pragma unroll
    for (int j = 0; j < dia_pat_nrun(PAT); j++) {
        const int c = row + a.off[kd];
#pragma unroll
        for (int q = 0; q < dia_pat_nq(PAT, j); q++) {
            const int p = CLAMP ? min(max(c + 2 * q, 0), a.ncols - 2) : c + 2 * q;
            dbl2_t v = *reinterpret_cast<const dbl2u_t *>(a.e.x + p);
            if constexpr (GM == SPMV_RESID0) v = *reinterpret_cast<const dbl2u_t *>(a.e.d + p) * v;
            if constexpr (CLAMP) {
                xv[vo + 2 * q] = c + 2 * q == p ? v.x : v.y;
                xv[vo + 2 * q + 1] = c + 2 * q + 1 == p ? v.x : v.y;
            } else {
                xv[vo + 2 * q] = v.x;
                xv[vo + 2 * q + 1] = v.y;
            }
        }
        kd += dia_pat_len(PAT, j);
        vo += 2 * dia_pat_nq(PAT, j);
    }
}

// CST (PAT 27, dia_constant): no codes; the interior coefficients from the
// arguments and the x operands of neighbours outside the grid taken as 0.0 (the
// coded rows hold the +0.0 code there: the same products up to the sign of a
// zero, added to an accumulator that is never -0.0 -- bitwise equal)
template <int MODE, int VB, int CW, int PAT, bool CST = false>
__global__ __launch_bounds__(256) void spmv_dia_pat_kernel(DiaArgs a) {
    constexpr bool DC = MODE == DIA_JACOBI_DC;
    constexpr int GM = DC ? SPMV_JACOBI : MODE;
    constexpr int NRUN = dia_pat_nrun(PAT), NV = dia_pat_nv(PAT);
    constexpr uint32_t MASK = (1u << VB) - 1;
    static_assert(dia_pat_k(PAT) * VB <= 32 * CW, "code words too short for the pattern");
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[DC ? 256 : 1];
    const double tv = (int)threadIdx.x < a.ntab ? a.vtab[threadIdx.x] : 0.0;
    double dv = 0.0;
    if constexpr (DC) dv = a.e.dt[threadIdx.x];
    int blk;
    if (a.band_bp > 0) {
        const int bb = a.band_bp >> 3, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        blk = (i / bb) * a.band_bp + x * bb + (i % bb);
    } else {
        blk = xcd_remap(blockIdx.x, gridDim.x);
    }
    const int row = a.row_begin + 512 * blk + 2 * (int)threadIdx.x;
    DiaEpi<MODE, false> ep;
    ep.load_codes(a.e, row, a.row_end);
    ep.load(a.e, row, a.row_end);
    uint32_t u[2 * CW];
    if constexpr (!CST) {
        const uint32_t *cp = a.codes + (int64_t)(min(row, a.row_end - 1) - a.code_row0) * CW;
#pragma unroll
        for (int q = 0; q < (2 * CW) / 4; q++) {
            const i32x4u_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4u_t *>(cp) + q);
#pragma unroll
            for (int j = 0; j < 4; j++) u[4 * q + j] = (uint32_t)v[j];
        }
        if constexpr ((2 * CW) % 4 >= 2) {
            const i32x2u_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x2u_t *>(cp + (2 * CW) / 4 * 4));
            u[(2 * CW) / 4 * 4] = (uint32_t)v.x;
            u[(2 * CW) / 4 * 4 + 1] = (uint32_t)v.y;
        }
        if constexpr ((2 * CW) % 2 == 1) u[2 * CW - 1] = __builtin_nontemporal_load(cp + 2 * CW - 1);
    }
    double xv[NV];
    // a block whose x runs all lie inside [0, ncols) (all but the first and last
    // plane or two of blocks) loads them unclamped: no selects, fewer registers
    const int rb = a.row_begin + 512 * blk;
    if (rb + a.off[0] >= 0 && rb + 511 + a.off[dia_pat_k(PAT) - 1] + 1 <= a.ncols - 1)
        dia_pat_loads<GM, PAT, false>(a, row, xv);
    else
        dia_pat_loads<GM, PAT, true>(a, row, xv);
    if ((int)threadIdx.x < a.ntab) stab[threadIdx.x] = tv;
    if constexpr (DC) sdt[threadIdx.x] = dv;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (row >= a.row_end) return;
    double acc0 = 0.0, acc1 = 0.0;
    if constexpr (CST) {
        static_assert(PAT == 27, "constant stencils: the 27-point pattern");
        const int q = row / a.gnx, gx = row - q * a.gnx;  // row even, nx even: the pair shares its grid row
        const int gz = q / a.gny, gy = q - gz * a.gny;
        const bool xlo = gx == 0, xhi = gx + 2 == a.gnx;
#pragma unroll
        for (int j = 0; j < 9; j++) {
            const int dz = j / 3 - 1, dy = j % 3 - 1;
            const bool ok = (unsigned)(gy + dy) < (unsigned)a.gny && (unsigned)(gz + dz) < (unsigned)a.gnz;
#pragma unroll
            for (int m = 0; m < 3; m++) {
                const int k = 3 * j + m;
                const double x0 = ok && !(m == 0 && xlo) ? xv[4 * j + m] : 0.0;
                const double x1 = ok && !(m == 2 && xhi) ? xv[4 * j + m + 1] : 0.0;
                acc0 = fma(a.cst[k], x0, acc0);
                acc1 = fma(a.cst[k], x1, acc1);
            }
        }
    } else {
        int kd = 0, vo = 0;
#pragma unroll
        for (int j = 0; j < NRUN; j++) {
#pragma unroll
            for (int m = 0; m < dia_pat_len(PAT, j); m++) {
                const int k = kd + m;
                acc0 = fma(stab[(u[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], xv[vo + m], acc0);
                acc1 = fma(stab[(u[CW + ((k * VB) >> 5)] >> ((k * VB) & 31)) & MASK], xv[vo + m + 1], acc1);
            }
            kd += dia_pat_len(PAT, j);
            vo += 2 * dia_pat_nq(PAT, j);
        }
    }
    ep.store(a.e, sdt, acc0, acc1);
}

// FAMG_DIA_CST=0: a constant 27-point stencil still reads its rows' codes
static bool dia_cst_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_CST");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_DIA_PAT=0: no DIA storage for more than 32 diagonals
static bool dia_pat_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_PAT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// The run pattern of a sorted offset list (0: none of the patterns above)
static int dia_pattern_of(const std::vector<int> &offs) {
    std::vector<int> len;
    for (size_t k = 0; k < offs.size(); k++) {
        if (k > 0 && offs[k] == offs[k - 1] + 1) len.back()++;
        else len.push_back(1);
    }
    for (int pat : {33, 27}) {
        if ((int)len.size() != dia_pat_nrun(pat)) continue;
        bool ok = true;
        for (int j = 0; ok && j < dia_pat_nrun(pat); j++) ok = len[j] == dia_pat_len(pat, j);
        if (ok) return pat;
    }
    return 0;
}

// One SGS color update with DIA codes of the color-permuted copy: stored row p
// (one per lane, rows of one color contiguous) is original row i = rowid[p];
// x[i] <- x[i] + d[p] (b[i] - sum_k a_k x[i + off_k]) in place (rows of one
// color never couple).  Loads branch-free as in spmv_dia_kernel; padding
// entries (code of +0.0) read a clamped in-range x and add exact zeros.
// NR > 0: nine runs of three consecutive offsets (27-point stencil), each run's
// x[c], x[c+1], x[c+2] from one 16-B and one 8-B load (18 loads instead of 32).
template <int VB, int CW, int NR = 0>
__global__ __launch_bounds__(256) void spmv_dia_sgs_kernel(DiaArgs a, const int32_t *rowid) {
    __shared__ double stab[VB == 4 ? 16 : 256];
    const double tv = (int)threadIdx.x < a.ntab ? a.vtab[threadIdx.x] : 0.0;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int p = a.row_begin + 256 * blk + (int)threadIdx.x;
    const int pc = min(p, a.row_end - 1);
    constexpr int KMAX = CW * 32 / VB < DIA_MAX ? CW * 32 / VB : DIA_MAX;
    constexpr uint32_t MASK = (1u << VB) - 1;
    uint32_t w[CW];
    const uint32_t *cp = a.codes + (int64_t)(pc - a.code_row0) * CW;
    if constexpr (CW == 1) {
        w[0] = __builtin_nontemporal_load(cp);
    } else if constexpr (CW == 2) {
        const i32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x2_t *>(cp));
        w[0] = (uint32_t)v.x;
        w[1] = (uint32_t)v.y;
    } else {
#pragma unroll
        for (int q = 0; q < CW / 4; q++) {
            const i32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t *>(cp) + q);
#pragma unroll
            for (int j = 0; j < 4; j++) w[4 * q + j] = (uint32_t)v[j];
        }
    }
    const int i = rowid[pc];
    const double xr = a.e.x[i], br = a.e.b[i], dr = a.e.d[pc];
    constexpr int KX = NR > 0 ? 3 * NR : KMAX;
    double xv[KX];
    if constexpr (NR > 0) {
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const int c = i + a.off[3 * j];
            const int p0 = min(max(c, 0), a.ncols - 2);
            const dbl2_t q = *reinterpret_cast<const dbl2u_t *>(a.e.x + p0);
            const double s2 = a.e.x[min(max(c + 2, 0), a.ncols - 1)];
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int t = c + u;
                xv[3 * j + u] = t == p0 ? q.x : t == p0 + 1 ? q.y : s2;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < KMAX; k++) xv[k] = a.e.x[min(max(i + a.off[k], 0), a.ncols - 1)];
    }
    if ((int)threadIdx.x < a.ntab) stab[threadIdx.x] = tv;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (p >= a.row_end) return;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < KX; k++) {
        const double f = fma(stab[(w[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], xv[k], acc);
        acc = (NR > 0 || k < a.k) ? f : acc;
    }
    a.e.y[i] = xr + dr * (br - acc);
}

// SpMM: Y = A X for up to SPMM_KB columns per launch (column-major X, Y with
// leading dimensions).  The slice is streamed once per column group; each
// (row, column) sum keeps the SpMV's order (ascending steps, fma), so every
// column is bitwise equal to a single-column SpMV.
constexpr int SPMM_KB = 8;

template <int CM, int KB>
__device__ __forceinline__ void spmm_step4(const char *__restrict__ blkp, int w, int k, bool paired,
                                           const int32_t *__restrict__ bs, int lane, int nu,
                                           const double *__restrict__ x, int64_t ldx, double (&acc)[KB]) {
    const char *ixb = blkp + (int64_t)w * SELL_VAL_STEP;
    double vv[4];
    int32_t cc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (u < nu) {
            const int t = k + u;
            const int64_t el = sell_elem(t, w, lane, paired);
            vv[u] = __builtin_nontemporal_load(reinterpret_cast<const double *>(blkp) + el);
            if constexpr (CM == 0) cc[u] = bs[t] + lane;
            else if constexpr (CM == 1)
                cc[u] = bs[t] + (int32_t)__builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(ixb) + el);
            else cc[u] = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(ixb) + el);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (u < nu) {
#pragma unroll
            for (int c = 0; c < KB; c++) acc[c] = fma(vv[u], x[cc[u] + c * ldx], acc[c]);
        }
    }
}

template <int CM, int KB>
__device__ __forceinline__ void spmm_walk(const char *blkp, bool paired, const int32_t *bs, int w, int lane,
                                          const double *x, int64_t ldx, double (&acc)[KB]) {
    for (int k = 0; k < w; k += 4) spmm_step4<CM, KB>(blkp, w, k, paired, bs, lane, min(4, w - k), x, ldx, acc);
}

template <int KB>
__global__ __launch_bounds__(256) void spmm_sell_kernel(SellArgs a, bool paired, int64_t ldx, double *y,
                                                        int64_t ldy) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int slice = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int row = a.row0[slice] + lane;
    const bool live = row < a.row0[slice + 1];
    const int t0 = a.soff[slice];
    const int w = a.soff[slice + 1] - t0;
    const uint32_t d = a.desc[slice];
    const char *blkp = a.data + (int64_t)(d & 0x3fffffffu) * 128;
    const int32_t *bs = a.base + t0;
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c] = 0.0;
    switch (d >> 30) {
    case 0: spmm_walk<0, KB>(blkp, paired, bs, w, lane, a.e.x, ldx, acc); break;
    case 1: spmm_walk<1, KB>(blkp, paired, bs, w, lane, a.e.x, ldx, acc); break;
    default: spmm_walk<2, KB>(blkp, paired, bs, w, lane, a.e.x, ldx, acc); break;
    }
    if (live) {
#pragma unroll
        for (int c = 0; c < KB; c++) y[row + c * ldy] = acc[c];
    }
}

// --------------------------------------------------------------------- vector

struct VecArgs {
    const int32_t *rowptr;
    const int32_t *col;     // int32 columns (O16 == false)
    const int16_t *off;     // col = row + off (O16)
    const double *val;      // fp64 values (VB == 0)
    const void *codes;      // 8 / 16-bit value codes (VB == 8 / 16) into vtab
    const double *vtab;
    int32_t row_begin, nrows;
    Epi e;
};

// Value and column of entry k (CSR order) for the wave-per-row kernel: fp64 or
// a code into the value table; int32 or a 16-bit offset from the row.
template <int VB, bool O16>
__device__ __forceinline__ void vec_entry(const VecArgs &a, int row, int k, double &v, int32_t &c) {
    if constexpr (VB == 0) v = __builtin_nontemporal_load(a.val + k);
    else if constexpr (VB == 8) v = a.vtab[__builtin_nontemporal_load(static_cast<const uint8_t *>(a.codes) + k)];
    else v = a.vtab[__builtin_nontemporal_load(static_cast<const uint16_t *>(a.codes) + k)];
    if constexpr (O16) c = row + (int32_t)__builtin_nontemporal_load(a.off + k);
    else c = __builtin_nontemporal_load(a.col + k);
}

// WPR waves per row (1, 2, 4): a level with few long rows (A_4 of the box
// hierarchies: 4096 rows of ~1400 entries, R_4: 512 rows) has too few waves
// to keep the loads in flight with one wave per row; with WPR > 1 the row's
// 64-entry chunks are dealt round-robin to its waves and the wave sums are
// added in LDS (a different lane split: the sum is bounded, not bitwise).
template <int MODE, int VB, bool O16, int WPR>
__global__ __launch_bounds__(256) void spmv_vector_kernel(VecArgs a) {
    __shared__ double part[4];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int wv = threadIdx.x >> 6;
    const int w = blk * (4 / WPR) + wv / WPR;
    const int sub = wv % WPR;
    if constexpr (WPR == 1)
        if (w >= a.nrows) return;
    const bool ok = w < a.nrows;
    const int row = a.row_begin + (ok ? w : 0);
    const int lane = threadIdx.x & 63;
    EpiOps<MODE> ep;
    if (ok && lane == 0 && sub == 0) ep.load(a.e, row);
    const int e0 = ok ? a.rowptr[row] : 0, e1 = ok ? a.rowptr[row + 1] : 0;
    constexpr int S = 64 * WPR;
    double acc = 0.0;
    int k = e0 + sub * 64 + lane;
    for (; k + 3 * S < e1; k += 4 * S) {
        double vv[4];
        int32_t cc[4];
#pragma unroll
        for (int u = 0; u < 4; u++) vec_entry<VB, O16>(a, row, k + S * u, vv[u], cc[u]);
        double xx[4];
#pragma unroll
        for (int u = 0; u < 4; u++) xx[u] = gx<MODE>(a.e, cc[u]);
#pragma unroll
        for (int u = 0; u < 4; u++) acc = fma(vv[u], xx[u], acc);
    }
    for (; k < e1; k += S) {
        double v;
        int32_t c;
        vec_entry<VB, O16>(a, row, k, v, c);
        acc = fma(v, gx<MODE>(a.e, c), acc);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if constexpr (WPR == 1) {
        if (lane == 0) ep.store(a.e, acc);
    } else {
        if (lane == 0) part[wv] = acc;
        __syncthreads();
        if (ok && lane == 0 && sub == 0) {
            double t = part[wv];
#pragma unroll
            for (int j = 1; j < WPR; j++) t += part[wv + j];
            ep.store(a.e, t);
        }
    }
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

// ---- SELL build: one wavefront per slice walks its rows in step order.

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, o));
    return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o));
    return v;
}

constexpr int64_t SELL_NONE = INT64_MAX;

// Walk the steps of one slice (all 64 lanes of the wave, uniform control flow).
// f(t, col, val, step_mode, step_base) per step; returns the step count, or -1
// if it would exceed max_steps.
template <bool ALIGNED, class F>
__device__ int sell_walk_build(const int64_t *rp, const int32_t *col, const double *val, int64_t row, bool live,
                               int64_t ncols, int max_steps, F &&f) {
    const int lane = threadIdx.x & 63;
    int64_t p = live ? rp[row] : 0;
    const int64_t e = live ? rp[row + 1] : 0;
    for (int t = 0;; t++) {
        bool real;
        if constexpr (ALIGNED) {
            const int64_t my = p < e ? (int64_t)col[p] - row : SELL_NONE;
            const int64_t m = wave_min64(my);
            if (m == SELL_NONE) return t;
            real = my == m;
        } else {
            real = p < e;
            if (!__any(real)) return t;
        }
        if (t >= max_steps) return -1;
        int64_t c = 0;
        double v = 0.0;
        if (real) { c = col[p]; v = val[p]; p++; }
        const int64_t b = wave_min64(real ? c - lane : SELL_NONE);
        if (!real) c = std::min<int64_t>(std::max<int64_t>(b + lane, 0), ncols - 1);
        const bool impl = __all(c == b + lane);
        const int64_t mn = wave_min64(c), mx = wave_max64(c);
        const int mode = impl ? 0 : (mx - mn < 65536 ? 1 : 2);
        f(t, c, v, mode, mode == 0 ? b : mn);
    }
}

__host__ __device__ inline int64_t sell_slice_bytes(int64_t w, int mode, int vb) {
    return sell_value_bytes(w, vb) + w * (mode == 0 ? 0 : mode == 1 ? 2 * SELL_C : 4 * SELL_C);
}

// ---- value table: the distinct fp64 bit patterns of a matrix (open
// addressing; stops counting past VT_MAX)
constexpr int VT_MAX = 65536;
constexpr int VT_SLOTS = 2 * VT_MAX;
constexpr unsigned long long VT_EMPTY = ~0ull;  // a NaN payload: a matrix holding it keeps fp64 values

__global__ __launch_bounds__(256) void k_value_set(const double *val, int64_t nnz, unsigned long long *slots,
                                                   unsigned int *cnt) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nnz; k += stride) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(val[k]);
        if (b == VT_EMPTY) {
            atomicAdd(cnt, (unsigned)VT_SLOTS);
            return;
        }
        unsigned h = (unsigned)((b * 0x9E3779B97F4A7C15ull) >> 47) & (VT_SLOTS - 1);
        for (int p = 0; p < VT_SLOTS; p++, h = (h + 1) & (VT_SLOTS - 1)) {
            unsigned long long cur = slots[h];
            if (cur == b) break;
            if ((cur == VT_EMPTY || p >= 16) && *(volatile unsigned *)cnt > (unsigned)VT_MAX) return;
            if (cur == VT_EMPTY) {
                cur = atomicCAS(&slots[h], VT_EMPTY, b);
                if (cur == VT_EMPTY) {
                    atomicAdd(cnt, 1u);
                    break;
                }
                if (cur == b) break;
            }
        }
    }
}

// Code width for m's values (0 = keep fp64, 4, 8 or 16) and the table: the
// distinct bit patterns, +0.0 (padding) included, ascending as unsigned.
static int value_table_of(const double *val, int64_t nnz, hipStream_t s, std::vector<unsigned long long> &tab,
                          unsigned *found = nullptr);

int csr_value_table(const GpuCsr &m, std::vector<unsigned long long> &tab);
static int value_table(const GpuCsr &m, std::vector<unsigned long long> &tab) { return csr_value_table(m, tab); }
int csr_value_table(const GpuCsr &m, std::vector<unsigned long long> &tab) {
    tab.clear();
    if (!g_value_codes || m.nnz == 0) return 0;
    return value_table_of(m.val.get(), m.nnz, m.ctx->stream, tab);
}

static int value_table_of(const double *val, int64_t nnz, hipStream_t s, std::vector<unsigned long long> &tab,
                          unsigned *found) {
    tab.clear();
    DevBuf<unsigned long long> slots(VT_SLOTS);
    DevBuf<unsigned int> cnt(1);
    FAMG_CHECK_HIP(hipMemsetAsync(slots.get(), 0xff, VT_SLOTS * sizeof(unsigned long long), s));
    FAMG_CHECK_HIP(hipMemsetAsync(cnt.get(), 0, sizeof(unsigned int), s));
    const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(nnz, 256));
    hipLaunchKernelGGL(k_value_set, dim3(grid), dim3(256), 0, s, val, nnz, slots.get(), cnt.get());
    FAMG_CHECK_HIP(hipGetLastError());
    std::vector<unsigned long long> h(VT_SLOTS);
    unsigned int c = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(h.data(), slots.get(), VT_SLOTS * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(&c, cnt.get(), sizeof(c), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (found) *found = c;  // distinct values present (the table adds 0.0)
    if (c > (unsigned)VT_MAX) return 0;
    for (unsigned long long b : h)
        if (b != VT_EMPTY) tab.push_back(b);
    if (std::find(tab.begin(), tab.end(), 0ull) == tab.end()) tab.push_back(0ull);
    std::sort(tab.begin(), tab.end());
    if ((int64_t)tab.size() > VT_MAX) {
        tab.clear();
        return 0;
    }
    return tab.size() <= 16 ? 4 : tab.size() <= 256 ? 8 : 16;
}

// plan[4 s ..] = {w_aligned (-1 = too wide), mode_aligned, w_plain, mode_plain}
__global__ __launch_bounds__(256) void k_sell_plan(const int64_t *rp, const int32_t *col, const double *val,
                                                   const int32_t *row0, int64_t nslices, int64_t ncols,
                                                   int max_steps, int32_t *plan) {
    const int64_t sl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sl >= nslices) return;
    const int64_t row = row0[sl] + (threadIdx.x & 63);
    const bool live = row < row0[sl + 1];
    int ma = 0, mp = 0;
    const int wa = sell_walk_build<true>(rp, col, val, row, live, ncols, max_steps,
                                         [&](int, int64_t, double, int m, int64_t) { ma = max(ma, m); });
    const int wp = sell_walk_build<false>(rp, col, val, row, live, ncols, max_steps,
                                          [&](int, int64_t, double, int m, int64_t) { mp = max(mp, m); });
    if ((threadIdx.x & 63) == 0) {
        plan[4 * sl + 0] = wa;
        plan[4 * sl + 1] = ma;
        plan[4 * sl + 2] = wp;
        plan[4 * sl + 3] = mp;
    }
}

// aligned[s] chooses the layout; desc/soff as uploaded; vb != 0: values as
// vb-bit codes into tab (ntab entries, ascending bit patterns)
__global__ __launch_bounds__(256) void k_sell_fill(const int64_t *rp, const int32_t *col, const double *val,
                                                   const int32_t *row0, const int32_t *soff, const uint32_t *desc,
                                                   const uint8_t *aligned, int64_t nslices, int64_t ncols,
                                                   bool paired, int vb, const unsigned long long *tab, int ntab,
                                                   int32_t *base, char *data) {
    const int64_t sl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sl >= nslices) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = row0[sl] + lane;
    const bool live = row < row0[sl + 1];
    const int w = soff[sl + 1] - soff[sl];
    const uint32_t d = desc[sl];
    const int smode = (int)(d >> 30);
    char *blkp = data + (int64_t)(d & 0x3fffffffu) * 128;
    char *ixb = blkp + sell_value_bytes(w, vb);
    double *vals = reinterpret_cast<double *>(blkp);
    int32_t *bs = base + soff[sl];
    unsigned long long cacc = 0;
    auto put = [&](int t, int64_t c, double v, int, int64_t b) {
        // the slice mode can exceed the step's: u16 steps use base = min column
        const int64_t sb = smode == 1 ? wave_min64(c) : b;
        const int64_t el = vb ? sell_group_elem(t, w, lane) : sell_elem(t, w, lane, paired);
        if (vb == 0) {
            vals[el] = v;
        } else {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
            int lo = 0, hi = ntab - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (tab[mid] < bits) lo = mid + 1;
                else hi = mid;
            }
            const int64_t unit = (int64_t)(t >> 3) * SELL_C + lane;
            if (vb == 16) {
                reinterpret_cast<uint16_t *>(blkp)[unit * 8 + (t & 7)] = (uint16_t)lo;
            } else {
                cacc |= (unsigned long long)lo << (vb * (t & 7));
                if ((t & 7) == 7 || t == w - 1) {
                    if (vb == 4) reinterpret_cast<uint32_t *>(blkp)[unit] = (uint32_t)cacc;
                    else reinterpret_cast<unsigned long long *>(blkp)[unit] = cacc;
                    cacc = 0;
                }
            }
        }
        if (lane == 0) bs[t] = smode == 2 ? 0 : (int32_t)sb;
        if (smode == 1) reinterpret_cast<uint16_t *>(ixb)[el] = (uint16_t)(c - sb);
        else if (smode == 2) reinterpret_cast<int32_t *>(ixb)[el] = (int32_t)c;
    };
    if (aligned[sl]) sell_walk_build<true>(rp, col, val, row, live, ncols, w, put);
    else sell_walk_build<false>(rp, col, val, row, live, ncols, w, put);
}

// ---- 8-bit codes of a vector (the Jacobi diagonal): table + codes, or 0
__global__ __launch_bounds__(256) void k_array_codes(const double *v, int64_t n, const unsigned long long *tab,
                                                     int ntab, uint8_t *code) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const unsigned long long bits = (unsigned long long)__double_as_longlong(v[i]);
    int lo = 0, hi = ntab - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tab[mid] < bits) lo = mid + 1;
        else hi = mid;
    }
    code[i] = (uint8_t)lo;
}

int64_t array_codes_u8(const double *v, int64_t n, Ctx &ctx, DevBuf<uint8_t> &code, DevBuf<double> &table,
                       double *dconst) {
    code.release();
    table.release();
    if (dconst) *dconst = 0.0;
    if (!g_value_codes || n == 0) return 0;
    std::vector<unsigned long long> tab;
    unsigned found = 0;
    const int vb = value_table_of(v, n, ctx.stream, tab, &found);
    if (vb != 4 && vb != 8) return 0;
    if (dconst && found == 1)  // one value present (the table's other entry is the added 0.0)
        for (unsigned long long bits : tab)
            if (bits != 0ull) std::memcpy(dconst, &bits, 8);
    table.resize(256);  // padded: kernels stage all 256 entries without a bound
    FAMG_CHECK_HIP(hipMemsetAsync(table.get(), 0, 256 * sizeof(double), ctx.stream));
    code.resize(n + 2);
    FAMG_CHECK_HIP(hipMemcpyAsync(table.get(), tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice,
                                  ctx.stream));
    FAMG_CHECK_HIP(hipMemsetAsync(code.get(), 0, n + 2, ctx.stream));
    hipLaunchKernelGGL(k_array_codes, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, ctx.stream, v, n,
                       reinterpret_cast<const unsigned long long *>(table.get()), (int)tab.size(), code.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(ctx.stream));
    return (int64_t)tab.size();
}

// ---- DIA build
constexpr int DIA_SLOTS = 256;
constexpr int DIA_EMPTY = INT32_MIN;

// rowid (optional): stored row p is the original row rowid[p] (a color-permuted
// SGS copy); offsets are taken against the original row
__global__ __launch_bounds__(256) void k_dia_offsets(const int64_t *rp, const int32_t *col, int64_t r0, int64_t r1,
                                                     const int32_t *rowid, int *slots, unsigned int *cnt) {
    const int64_t i = r0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= r1) return;
    const int64_t ri = rowid ? rowid[i] : i;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        const int64_t o64 = (int64_t)col[e] - ri;
        if (o64 <= INT32_MIN / 2 || o64 >= INT32_MAX / 2) {
            atomicAdd(cnt, (unsigned)DIA_SLOTS);
            return;
        }
        const int o = (int)o64;
        unsigned h = ((unsigned)o * 2654435761u) >> 24;
        for (int p = 0; p < DIA_SLOTS; p++, h = (h + 1) & (DIA_SLOTS - 1)) {
            int cur = slots[h];
            if (cur == o) break;
            if ((cur == DIA_EMPTY || p >= 8) && *(volatile unsigned *)cnt > (unsigned)DIA_MAX) return;
            if (cur == DIA_EMPTY) {
                cur = atomicCAS(&slots[h], DIA_EMPTY, o);
                if (cur == DIA_EMPTY) {
                    atomicAdd(cnt, 1u);
                    break;
                }
                if (cur == o) break;
            }
        }
    }
}

// codes of row i (rows >= n: padding, all +0.0)
__global__ __launch_bounds__(256) void k_dia_fill(const int64_t *rp, const int32_t *col, const double *val,
                                                  int64_t r0, int64_t r1, int64_t nrows_alloc, const int32_t *rowid,
                                                  DiaArgs off, int vb, int cw, const unsigned long long *tab, int ntab,
                                                  int zero_code, uint32_t *codes) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nrows_alloc) return;
    const int64_t i = r0 + j;
    int c[DIA_MAX];
    for (int k = 0; k < off.k; k++) c[k] = zero_code;
    if (i < r1) {
        const int64_t ri = rowid ? rowid[i] : i;
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int o = (int)((int64_t)col[e] - ri);
            int k = 0;
            while (off.off[k] != o) k++;
            const unsigned long long bits = (unsigned long long)__double_as_longlong(val[e]);
            int lo = 0, hi = ntab - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (tab[mid] < bits) lo = mid + 1;
                else hi = mid;
            }
            c[k] = lo;
        }
    }
    for (int q = 0; q < cw; q++) {
        uint32_t wd = 0;
        for (int k = 0; k < off.k; k++)
            if ((k * vb) >> 5 == q) wd |= (uint32_t)c[k] << ((k * vb) & 31);
        codes[j * cw + q] = wd;
    }
}

// DIA codes storage for rows [r0, r1) of m (auto policy, square, >= SELL_MIN_ROWS
// rows, 4/8-bit value table, <= DIA_MAX diagonals filled to >= 80 %).  Returns
// true if built.
static bool build_dia(GpuCsr &m, int vb, const std::vector<unsigned long long> &tab,
                      const std::vector<int64_t> &rp, int64_t r0, int64_t r1, const int32_t *rowid = nullptr) {
    const int64_t nr = r1 - r0;
    // a rectangular matrix qualifies only through a row segment (the halo
    // interior of a distributed level: [owned | ghost] columns); every stored
    // entry's column is row + off, so only padding entries are clamped
    const bool square_or_segment = m.nrows == m.ncols || (m.seg_rows.size() > 2 && m.ncols >= m.nrows);
    if (g_spmv_format_policy != 0 || (vb != 4 && vb != 8) || !square_or_segment || nr < SELL_MIN_ROWS ||
        m.ncols >= (int64_t(1) << 30))
        return false;
    hipStream_t s = m.ctx->stream;
    DevBuf<int> slots(DIA_SLOTS);
    DevBuf<unsigned int> cnt(1);
    std::vector<int> hs(DIA_SLOTS, DIA_EMPTY);
    FAMG_CHECK_HIP(hipMemcpyAsync(slots.get(), hs.data(), DIA_SLOTS * sizeof(int), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemsetAsync(cnt.get(), 0, sizeof(unsigned int), s));
    hipLaunchKernelGGL(k_dia_offsets, dim3((unsigned)ceil_div(nr, 256)), dim3(256), 0, s, m.rp64.get(),
                       m.col.get(), r0, r1, rowid, slots.get(), cnt.get());
    FAMG_CHECK_HIP(hipGetLastError());
    unsigned int c = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(hs.data(), slots.get(), DIA_SLOTS * sizeof(int), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(&c, cnt.get(), sizeof(c), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (c > (unsigned)DIA_MAX) return false;
    std::vector<int> offs;
    for (int o : hs)
        if (o != DIA_EMPTY) offs.push_back(o);
    std::sort(offs.begin(), offs.end());
    const int K = (int)offs.size();
    if (K == 0 || (int64_t)K * nr * 4 > (rp[r1] - rp[r0]) * 5) return false;  // >= 80 % filled
    // more than 32 diagonals: only a run pattern's kernel (no SGS sweep)
    const int pat = K > 32 && dia_pat_enabled() ? dia_pattern_of(offs) : 0;
    if (K > 32 && (rowid || pat == 0)) return false;
    const int bits = K * vb;
    int cw = 1;
    if (pat) cw = (bits + 31) / 32;
    else
        while (cw * 32 < bits) cw *= 2;
    DiaArgs oa{};
    oa.k = K;
    for (int k = 0; k < K; k++) oa.off[k] = offs[k];
    const int zero_code = (int)(std::lower_bound(tab.begin(), tab.end(), 0ull) - tab.begin());
    const int64_t nalloc = nr + 2;
    m.dia_codes.resize(nalloc * cw);
    m.dia_vtab.resize(tab.size());
    FAMG_CHECK_HIP(hipMemcpyAsync(m.dia_vtab.get(), tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_dia_fill, dim3((unsigned)ceil_div(nalloc, 256)), dim3(256), 0, s, m.rp64.get(), m.col.get(),
                       m.val.get(), r0, r1, nalloc, rowid, oa, vb, cw,
                       reinterpret_cast<const unsigned long long *>(m.dia_vtab.get()), (int)tab.size(), zero_code,
                       m.dia_codes.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.dia_k = K;
    m.dia_cw = cw;
    m.dia_off = offs;
    m.dia_r0 = r0;
    m.dia_r1 = r1;
    m.dia_vbits = vb;
    m.dia_ntab = (int64_t)tab.size();
    m.dia_rowid = rowid;
    m.dia_pat = pat;
    return true;
}

// DIA codes of a color-permuted SGS copy (rows grouped by color, columns in the
// original numbering): diagonals are col - rowid[p].  Used only by the SGS
// sweep; the copy's other storage stays as chosen.
bool build_dia_sgs(GpuCsr &m, const int32_t *rowid) {
    if (g_spmv_format_policy != 0 || !g_value_codes || m.nrows == 0 || m.nrows != m.ncols) return false;
    std::vector<int64_t> rp(m.nrows + 1);
    FAMG_CHECK_HIP(hipMemcpyAsync(rp.data(), m.rp64.get(), (m.nrows + 1) * sizeof(int64_t), hipMemcpyDeviceToHost,
                                  m.ctx->stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(m.ctx->stream));
    std::vector<unsigned long long> tab;
    const int vb = value_table(m, tab);
    DevBuf<uint32_t> keep_codes = std::move(m.dia_codes);  // a segment DIA the finalize may have built
    DevBuf<double> keep_tab = std::move(m.dia_vtab);
    if (!build_dia(m, vb, tab, rp, 0, m.nrows, rowid)) {
        m.dia_codes = std::move(keep_codes);
        m.dia_vtab = std::move(keep_tab);
        m.dia_rowid = nullptr;
        return false;
    }
    m.dia_seg = -2;  // not a row segment of the plain SpMV
    return true;
}

void build_sell(GpuCsr &m, const std::vector<int64_t> &rp) {
    m.sell_row0.release();
    m.sell_soff.release();
    m.sell_desc.release();
    m.sell_base.release();
    m.sell_data.release();
    m.sell_vtab.release();
    m.dia_codes.release();
    m.dia_vtab.release();
    m.dia_ntab = 0;
    m.dia_k = m.dia_cw = m.dia_vbits = m.dia_pat = 0;
    m.dia_r0 = m.dia_r1 = m.dia_seg = 0;
    m.dia_rowid = nullptr;
    m.dia_off.clear();
    m.nslices = m.sell_steps = m.sell_bytes = m.sell_ntab = 0;
    m.sell_vbits = 0;
    m.sell_mode_slices[0] = m.sell_mode_slices[1] = m.sell_mode_slices[2] = 0;
    m.sell_short = false;
    m.seg_slc.clear();
    const int pol = g_spmv_format_policy;
    if (pol == 1 || pol == 3 || m.kind_pin >= 1 || m.nrows == 0 || m.nnz == 0) return;
    // slices never straddle a segment
    std::vector<int32_t> row0;
    std::vector<int64_t> seg_slc{0};
    int64_t maxlen = 0;
    for (size_t g = 0; g + 1 < m.seg_rows.size(); g++) {
        for (int64_t r0 = m.seg_rows[g]; r0 < m.seg_rows[g + 1]; r0 += SELL_C) row0.push_back((int32_t)r0);
        seg_slc.push_back((int64_t)row0.size());
    }
    for (int64_t r = 0; r < m.nrows; r++) maxlen = std::max<int64_t>(maxlen, rp[r + 1] - rp[r]);
    const int max_w = pol == 2 ? 256 : SELL_MAX_W;
    if (maxlen > max_w) return;
    row0.push_back((int32_t)m.nrows);
    const int64_t ns = (int64_t)row0.size() - 1;
    std::vector<unsigned long long> tab;
    const int vb = value_table(m, tab);
    // DIA codes on the whole matrix, or (several row segments: the halo
    // interior of a distributed level) on its longest segment beside SELL
    int64_t dseg = 0;
    for (size_t g = 1; g + 1 < m.seg_rows.size(); g++)
        if (m.seg_rows[g + 1] - m.seg_rows[g] > m.seg_rows[dseg + 1] - m.seg_rows[dseg]) dseg = (int64_t)g;
    // (a renumbered copy, reorder.hip, keeps its rows' stored order: no DIA, no aligned slices)
    if (!m.order_fixed && build_dia(m, vb, tab, rp, m.seg_rows[dseg], m.seg_rows[dseg + 1])) {
        m.dia_seg = dseg;
        if (m.dia_r0 == 0 && m.dia_r1 == m.nrows) return;
    }
    hipStream_t s = m.ctx->stream;
    DevBuf<int32_t> drow0(ns + 1), dplan(4 * ns);
    FAMG_CHECK_HIP(hipMemcpyAsync(drow0.get(), row0.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const dim3 grid((unsigned)ceil_div(ns, 4));
    hipLaunchKernelGGL(k_sell_plan, grid, dim3(256), 0, s, m.rp64.get(), m.col.get(), m.val.get(), drow0.get(), ns,
                       m.ncols, max_w, dplan.get());
    FAMG_CHECK_HIP(hipGetLastError());
    std::vector<int32_t> plan(4 * ns);
    FAMG_CHECK_HIP(hipMemcpyAsync(plan.data(), dplan.get(), plan.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    // per slice: the cheaper layout; then offsets
    std::vector<int32_t> soff(ns + 1, 0);
    std::vector<uint32_t> desc(ns);
    std::vector<uint8_t> aligned(ns);
    int64_t bytes = 0, steps = 0, cnt[3] = {0, 0, 0};
    for (int64_t k = 0; k < ns; k++) {
        const int wa = plan[4 * k], ma = plan[4 * k + 1], wp = plan[4 * k + 2], mp = plan[4 * k + 3];
        const bool al = !m.order_fixed && wa >= 0 && sell_slice_bytes(wa, ma, vb) <= sell_slice_bytes(wp, mp, vb);
        const int w = al ? wa : wp, md = al ? ma : mp;
        aligned[k] = al;
        if (bytes / 128 >= (int64_t(1) << 30) || steps + w >= (int64_t(1) << 31)) return;
        desc[k] = (uint32_t)(bytes / 128) | ((uint32_t)md << 30);
        bytes += sell_slice_bytes(w, md, vb);
        steps += w;
        soff[k + 1] = (int32_t)steps;
        cnt[md]++;
    }
    // auto: SELL pays when there are enough slices to fill the chip (>= 1024
    // slices = 64K rows) and it streams no more than 1.25x the CSR bytes;
    // measured on the 256^3 hierarchy (scripts/ab_levels.py).
    const bool ok = pol == 2 || m.kind_pin == 0 || (bytes * 100 <= 12 * m.nnz * 125 && (m.nrows >= SELL_MIN_ROWS || maxlen <= 16) &&
                                 (vec_min_avg() >= VECTOR_MIN_AVG || m.nnz < vec_min_avg() * m.nrows));
    if (!ok) return;
    m.sell_row0 = std::move(drow0);
    m.sell_soff.resize(ns + 1);
    m.sell_desc.resize(ns);
    m.sell_base.resize(std::max<int64_t>(1, steps));
    m.sell_data.resize(std::max<int64_t>(128, bytes));
    DevBuf<uint8_t> dal(ns);
    const char *lay = getenv("FAMG_SELL_LAYOUT");
    m.sell_paired = !(lay && std::string(lay) == "step");
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_soff.get(), soff.data(), (ns + 1) * sizeof(int32_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_desc.get(), desc.data(), ns * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(dal.get(), aligned.data(), ns, hipMemcpyHostToDevice, s));
    if (vb) {
        m.sell_vtab.resize(tab.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_vtab.get(), tab.data(), tab.size() * sizeof(double),
                                      hipMemcpyHostToDevice, s));
    }
    hipLaunchKernelGGL(k_sell_fill, grid, dim3(256), 0, s, m.rp64.get(), m.col.get(), m.val.get(),
                       m.sell_row0.get(), m.sell_soff.get(), m.sell_desc.get(), dal.get(), ns, m.ncols,
                       m.sell_paired, vb, reinterpret_cast<const unsigned long long *>(m.sell_vtab.get()),
                       (int)tab.size(), m.sell_base.get(), m.sell_data.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.nslices = ns;
    m.sell_steps = steps;
    m.sell_bytes = bytes;
    m.sell_vbits = vb;
    m.sell_ntab = vb ? (int64_t)tab.size() : 0;
    for (int k = 0; k < 3; k++) m.sell_mode_slices[k] = cnt[k];
    m.seg_slc = seg_slc;
    // short slices (coded, <= 4 steps, implicit / u16 columns, pairs of equal
    // width and column mode, one row segment): spmv_sell_short_kernel
    bool sh = vb != 0 && ns % 2 == 0 && cnt[2] == 0 && m.seg_rows.size() == 2;
    for (int64_t k = 0; sh && k < ns; k += 2) {
        const int32_t wa = soff[k + 1] - soff[k], wb = soff[k + 2] - soff[k + 1];
        sh = wa <= 4 && wa == wb && (desc[k] >> 30) == (desc[k + 1] >> 30) && row0[k + 1] - row0[k] == 64;
    }
    m.sell_short = sh;
}

// ---- wave-per-row storage: value codes (8/16-bit) and 16-bit row offsets
__global__ __launch_bounds__(256) void k_vec_maxoff(const int64_t *rp, const int32_t *col, int64_t n,
                                                    unsigned long long *mx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    unsigned long long m = 0;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        const int64_t o = (int64_t)col[e] - i;
        const unsigned long long a = (unsigned long long)(o < 0 ? -o : o);
        m = a > m ? a : m;
    }
    atomicMax(mx, m);
}

__global__ __launch_bounds__(256) void k_vec_fill(const int64_t *rp, const int32_t *col, const double *val, int64_t n,
                                                  int vb, const unsigned long long *tab, int ntab, bool o16,
                                                  void *codes, int16_t *off) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        if (o16) off[e] = (int16_t)((int64_t)col[e] - i);
        if (vb) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(val[e]);
            int lo = 0, hi = ntab - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (tab[mid] < bits) lo = mid + 1;
                else hi = mid;
            }
            if (vb == 8) static_cast<uint8_t *>(codes)[e] = (uint8_t)lo;
            else static_cast<uint16_t *>(codes)[e] = (uint16_t)lo;
        }
    }
}

static void build_vec_codes(GpuCsr &m) {
    m.vec_codes.release();
    m.vec_off.release();
    m.vec_vbits = 0;
    m.vec_o16 = false;
    if (m.nnz == 0) return;
    hipStream_t s = m.ctx->stream;
    std::vector<unsigned long long> tab;
    int vb = value_table(m, tab);
    if (vb == 4) vb = 8;
    DevBuf<unsigned long long> mx(1);
    FAMG_CHECK_HIP(hipMemsetAsync(mx.get(), 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_vec_maxoff, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s, m.rp64.get(),
                       m.col.get(), m.nrows, mx.get());
    unsigned long long hmx = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&hmx, mx.get(), sizeof(hmx), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    const bool o16 = g_value_codes && hmx <= 32767;
    if (!vb && !o16) return;
    if (vb) {
        m.sell_vtab.resize(tab.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sell_vtab.get(), tab.data(), tab.size() * sizeof(double),
                                      hipMemcpyHostToDevice, s));
        m.vec_codes.resize(m.nnz * (vb / 8));
    }
    if (o16) m.vec_off.resize(m.nnz);
    hipLaunchKernelGGL(k_vec_fill, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s, m.rp64.get(), m.col.get(),
                       m.val.get(), m.nrows, vb, reinterpret_cast<const unsigned long long *>(m.sell_vtab.get()),
                       (int)tab.size(), o16, (void *)m.vec_codes.get(), m.vec_off.get());
    FAMG_CHECK_HIP(hipGetLastError());
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.vec_vbits = vb;
    m.vec_o16 = o16;
    m.sell_ntab = vb ? (int64_t)tab.size() : 0;
}

static int vec_waves_per_row(int64_t rows, int64_t nnz);

void choose_kernel(GpuCsr &m) {
    if (m.has_dia() && !m.dia_rowid && m.dia_r0 == 0 && m.dia_r1 == m.nrows) m.kernel = SPMV_KERNEL_DIA;
    else if (m.has_bsr()) m.kernel = SPMV_KERNEL_BSR;
    else if (m.kind_pin == 1) {  // a renumbered copy of a wave-per-row matrix (reorder.hip)
        m.kernel = SPMV_KERNEL_VECTOR;
        m.vec_wpr = vec_waves_per_row(m.nrows, m.nnz);
        build_vec_codes(m);
    }
    else if (m.kind_pin == 2) m.kernel = SPMV_KERNEL_STREAM;
    else if (m.has_scs() && m.scs_seg < 0) m.kernel = SPMV_KERNEL_SCS;
    else if (m.has_sellp()) m.kernel = SPMV_KERNEL_SELLP;
    else if (m.has_xs()) m.kernel = SPMV_KERNEL_XS;
    else if (m.has_sell()) m.kernel = SPMV_KERNEL_SELL;
    else if (g_spmv_format_policy == 3 ||
             (g_spmv_format_policy == 0 && m.nrows > 0 && m.nnz >= vec_min_avg() * m.nrows)) {
        m.kernel = SPMV_KERNEL_VECTOR;
        m.vec_wpr = vec_waves_per_row(m.nrows, m.nnz);
        build_vec_codes(m);
    }
    else m.kernel = SPMV_KERNEL_STREAM;
}

// ------------------------------------------------------------------ dispatch

// KERNEL<MODE [, extra template args]> on (grid, block, stream s); the optional
// trailing argument is pasted after MODE (e.g. FAMG_LAY1).
#define FAMG_LAUNCH_MODES(KERNEL, grid, block, s, args, ...)                             \
    switch (mode) {                                                                     \
    case SPMV_SET: KERNEL<SPMV_SET __VA_ARGS__><<<grid, block, 0, s>>>(args); break;       \
    case SPMV_ADD: KERNEL<SPMV_ADD __VA_ARGS__><<<grid, block, 0, s>>>(args); break;       \
    case SPMV_RESID: KERNEL<SPMV_RESID __VA_ARGS__><<<grid, block, 0, s>>>(args); break;   \
    case SPMV_JACOBI: KERNEL<SPMV_JACOBI __VA_ARGS__><<<grid, block, 0, s>>>(args); break; \
    case SPMV_SGS: KERNEL<SPMV_SGS __VA_ARGS__><<<grid, block, 0, s>>>(args); break;       \
    case SPMV_RESID0: KERNEL<SPMV_RESID0 __VA_ARGS__><<<grid, block, 0, s>>>(args); break; \
    case SPMV_ADD0: KERNEL<SPMV_ADD0 __VA_ARGS__><<<grid, block, 0, s>>>(args); break;     \
    default: break;                                                                     \
    }
#define FAMG_VEC(VB, O16, W) , VB, O16, W

// waves per row of the wave-per-row kernel: few long rows get 2 or 4 waves each.
// Chosen once per matrix at finalize from all of its rows, so every row segment
// (halo interior / boundary launches, rank-local copies) splits its rows the
// same way; flag FLAG_VEC_WPR (FAMG_VEC_WPR, amg_set_flag) forces 1/2/4.
static int vec_waves_per_row(int64_t rows, int64_t nnz) {
    const int64_t avg = nnz / std::max<int64_t>(1, rows);
    if (rows <= 16384 && avg >= 512) return 4;
    if (rows <= 65536 && avg >= 256) return 2;
    return 1;
}
#define FAMG_LAY0 , 0
#define FAMG_LAY1 , 1
#define FAMG_LAY4 , 4
#define FAMG_LAY8 , 8
#define FAMG_LAY16 , 16

void spmm(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k, hipStream_t s) {
    if (spmm_compressed(m, x, ldx, y, ldy, k, s)) return;  // DIA codes, stencil classes, 3x3 blocks (spmm.hip)
    if (m.kernel != SPMV_KERNEL_SELL || m.sell_vbits) {  // other storages: one SpMV per column
        for (int64_t c = 0; c < k; c++) spmv(m, x + c * ldx, y + c * ldy, SPMV_SET, SpmvEpi{}, s);
        return;
    }
    if (m.nslices == 0) return;
    const dim3 grid((unsigned)ceil_div(m.nslices, 4)), block(256);
    for (int64_t c0 = 0; c0 < k; c0 += SPMM_KB) {
        const int kb = (int)std::min<int64_t>(SPMM_KB, k - c0);
        Epi e{x + c0 * ldx, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        SellArgs a{m.sell_row0.get(), m.sell_soff.get(), m.sell_desc.get(), m.sell_base.get(),
                   m.sell_data.get(), 0, (int32_t)m.nslices, e, nullptr, 0, 1};
        double *yc = y + c0 * ldy;
        switch (kb) {
        case 1: hipLaunchKernelGGL(spmm_sell_kernel<1>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 2: hipLaunchKernelGGL(spmm_sell_kernel<2>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 3: hipLaunchKernelGGL(spmm_sell_kernel<3>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 4: hipLaunchKernelGGL(spmm_sell_kernel<4>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 5: hipLaunchKernelGGL(spmm_sell_kernel<5>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 6: hipLaunchKernelGGL(spmm_sell_kernel<6>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        case 7: hipLaunchKernelGGL(spmm_sell_kernel<7>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        default: hipLaunchKernelGGL(spmm_sell_kernel<8>, grid, block, 0, s, a, m.sell_paired, ldx, yc, ldy); break;
        }
        FAMG_CHECK_HIP(hipGetLastError());
    }
}

template <int M, int VB, int CW>
static void launch_dia(int runs, bool nt, dim3 grid, dim3 block, hipStream_t s, const DiaArgs &a, bool cst = false) {
    if constexpr (CW * 32 / VB >= 7) {
        if (runs == -1 && cst) {  // constant 7-point stencil: no codes
            if constexpr (M != DIA_JACOBI_DC && M != DIA_RESID0_DC) {
                // auto (0): two pairs for SET (the solve loops' operator apply: 52.3 -> 49.0 us on
                // 256^3), one for the cycle's RESID0 / JACOBI (in-cycle 65.9 -> 74.3 and
                // 84.6 -> 89.4 us with two: profiles/r05/ab_dia7_rp.txt)
                int rp = (int)flag(FLAG_DIA7_RP);
                if (rp == 0) rp = M == SPMV_SET ? 2 : 1;
                if (rp > 1 && (a.band_bp == 0 || a.band_bp % (8 * rp) == 0)) {
                    const dim3 g((unsigned)ceil_div((int64_t)grid.x, rp));
                    if (rp == 2) spmv_dia7c_kernel<M, 2><<<g, block, 0, s>>>(a);
                    else spmv_dia7c_kernel<M, 4><<<g, block, 0, s>>>(a);
                    return;
                }
            }
            spmv_dia_kernel<M, VB, CW, false, -1, true><<<grid, block, 0, s>>>(a);
            return;
        }
    }
    if constexpr (M == DIA_JACOBI_DK || M == DIA_RESID0_DK) {  // chosen only for the 7-point run kernel
        if constexpr (CW * 32 / VB >= 7) {
            if (runs == -1) {
                spmv_dia_kernel<M, VB, CW, false, -1><<<grid, block, 0, s>>>(a);
                return;
            }
        }
        fail(AMG_ERR_INVALID, "DIA: constant-diagonal epilogue outside the 7-point run kernel");
    } else {
    if constexpr (CW * 32 / VB >= 27) {
        if (runs == 9) {
            spmv_dia_kernel<M, VB, CW, false, 9><<<grid, block, 0, s>>>(a);
            return;
        }
    }
    if constexpr (CW * 32 / VB >= 7) {
        if (runs == -1) {
            spmv_dia_kernel<M, VB, CW, false, -1><<<grid, block, 0, s>>>(a);
            return;
        }
    }
    if (nt) spmv_dia_kernel<M, VB, CW, true><<<grid, block, 0, s>>>(a);
    else spmv_dia_kernel<M, VB, CW, false><<<grid, block, 0, s>>>(a);
    }
}

// A/B switch FAMG_DIA_RUNS=0: the 27-point DIA kernels load every diagonal's pair
static bool dia_runs() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_RUNS");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_SELL_SHORT=0: short-slice operators take the generic SELL kernel
static bool sell_short_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_SELL_SHORT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_DIA_PAT27=0: the 27-point DIA SpMV takes spmv_dia_kernel<NR = 9>
static bool dia_pat27() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_PAT27");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_DIA_RC=0: the folded DIA residual gathers 8-B values of d
static bool dia_rc_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_RC");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_DIA_RUNS7=0: the 7-point DIA kernels load every diagonal's pair
static bool dia_runs7() {
    static const bool on = [] {
        const char *e = getenv("FAMG_DIA_RUNS7");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B switch FAMG_DIA_DK=0 / amg_set_flag(1, 0): a constant coded diagonal is still read per row
static bool dia_dk_enabled() { return flag(FLAG_DIA_DK) != 0; }

// The 7-point run pattern of the DIA kernel (NR = -1)
static bool dia_run7(const GpuCsr &m) {
    return m.dia_k == 7 && dia_runs7() && m.dia_off[3] == m.dia_off[2] + 1 && m.dia_off[4] == m.dia_off[2] + 2;
}

// JACOBI / RESID0 with a coded diagonal of one value on the 7-point DIA kernel:
// d is dt[0], no codes are read
static bool dia_dk(const GpuCsr &m, const SpmvEpi &epi) {
    return epi.dc && epi.dk != 0.0 && dia_dk_enabled() && !m.dia_pat && dia_run7(m);
}

bool dia7_cst_dk(const GpuCsr &m, const SpmvEpi &epi) {
    return m.kernel == SPMV_KERNEL_DIA && m.dia_cst && m.dia_k == 7 && dia_cst_enabled() && dia_dk(m, epi) &&
           m.dia_vbits > 0 && m.dia_cw * 32 / m.dia_vbits >= 7 &&
           m.nrows == (int64_t)m.dia_cst_n[0] * m.dia_cst_n[1] * m.dia_cst_n[2];
}

thread_local LaunchLog *g_launch_log = nullptr;

// Launch-plan record of one spmv() call (amg_multigrid_cycle_plan): the storage
// the dispatch below takes, the bytes that storage streams for the launched rows,
// x read once, and the epilogue's vector traffic per mode.
static void log_spmv(const GpuCsr &m, SpmvMode mode, const SpmvEpi &epi, int64_t seg) {
    const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg], r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
    const int64_t r = r1 - r0;
    if (r <= 0 || m.nrows <= 0) return;
    const double frac = (double)r / (double)m.nrows;
    auto part = [&](int64_t whole) { return seg < 0 ? whole : (int64_t)std::llround((double)whole * frac); };
    int kernel = m.kernel;
    const char *name = "csr-stream";
    int64_t mat = 0;
    const int64_t csr_mat = part(m.index_bytes());
    const int64_t dia_bytes = 4 * (int64_t)m.dia_cw * r + 8 * m.dia_ntab;
    if (m.gtx_on && (seg < 0 || m.rframe.on()) && gtx_supports(m, mode)) {
        kernel = SPMV_KERNEL_GTC;
        name = "gtx";
        mat = 2 * part(m.nrows) + 12 * m.gtx_nent + 8 * m.gtx_nclass;
    } else if (m.gtc_on && (seg < 0 || m.rframe.on()) && gtc_supports(m, mode)) {
        kernel = SPMV_KERNEL_GTC;
        name = "gtc";
        mat = part(m.nrows) + 2 * (int64_t)m.gtc_nce + 8 * (int64_t)m.gtc_ntab;
    } else if (m.kernel == SPMV_KERNEL_BSR) {
        name = "bsr3";
        mat = part(m.stream_bytes());
    } else if (m.kernel == SPMV_KERNEL_SCS || (m.has_scs() && seg >= 0 && seg == m.scs_seg && mode != SPMV_SGS)) {
        kernel = SPMV_KERNEL_SCS;
        name = (m.xscs && (seg < 0 || m.cframe.on())) ? "xscs" : m.scs_lanes ? "scs_lanes" : "scs";
        mat = m.scs_ib * r + 8 * m.scs_k * m.scs_nclass + 4 * m.scs_k;
    } else if (m.kernel == SPMV_KERNEL_XS && seg < 0 && xs_supports(mode)) {
        name = "xsell";
        mat = m.stream_bytes();
    } else if (m.kernel == SPMV_KERNEL_SELLP) {
        name = "sellp";
        mat = part(m.stream_bytes());
    } else if (mode == SPMV_SGS && m.has_dia() && m.dia_rowid) {
        kernel = SPMV_KERNEL_DIA;
        name = "dia_sgs";
        mat = dia_bytes;
    } else if (m.kernel == SPMV_KERNEL_DIA || (m.has_dia() && !m.dia_rowid && seg >= 0 && seg == m.dia_seg)) {
        kernel = SPMV_KERNEL_DIA;
        name = (m.dia_pat || (m.dia_k == 27 && dia_runs() && dia_pat27())) ? "dia_pat" : "dia";
        mat = (m.dia_cst && seg < 0) ? (int64_t)m.dia_k * 8 : dia_bytes;  // constant stencil: no codes read
    } else if (m.kernel == SPMV_KERNEL_SELL) {
        name = (m.sell_short && seg < 0 && mode != SPMV_SGS && mode != SPMV_RESID0 && sell_short_enabled())
                   ? "sell_short" : "sell";
        mat = part(m.stream_bytes());
    } else if (m.kernel == SPMV_KERNEL_VECTOR) {
        name = "vector";
        mat = part(m.stream_bytes());
    } else {
        kernel = SPMV_KERNEL_STREAM;
        mat = csr_mat;
    }
    const int64_t xcols = part(m.ncols);
    const bool dk = (kernel == SPMV_KERNEL_DIA && dia_dk(m, epi)) ||  // one value of d: no codes read
                    (kernel == SPMV_KERNEL_GTC && (mode == SPMV_ADD0 || mode == SPMV_SETDF) && epi.dc && epi.dk != 0.0 &&
                     dia_dk_enabled());
    const int64_t db = dk ? 0 : (epi.dc ? 1 : 8);  // bytes per diagonal entry (8-bit codes or fp64)
    int64_t vec = 8 * xcols;              // x read once
    switch (mode) {
    case SPMV_SET: vec += 8 * r; break;                  // y written
    case SPMV_ADD: vec += 16 * r; break;                 // y read + written
    case SPMV_RESID: vec += 16 * r; break;               // b read, y written
    case SPMV_JACOBI: vec += 16 * r + db * r; break;     // b, d read, y written
    case SPMV_SGS: vec += 28 * r; break;                 // perm, d, b read, x written
    case SPMV_RESID0:  // x = b; d gathered beside x (1-B codes in the DIA and x-staged class kernels); y written
        vec += 8 * r + (dk ? 0 : (((kernel == SPMV_KERNEL_DIA && dia_rc_enabled()) || (kernel == SPMV_KERNEL_SCS && m.xscs))
                                   && epi.dc ? 1 : 8)) * xcols;
        break;
    case SPMV_ADD0: vec += 16 * r + db * r; break;       // b, d read, y written
    case SPMV_SETDF: vec += 16 * r + db * r; break;      // y and d*y written, d read
    }
    log_launch(name, kernel, mode, r, mat + vec, csr_mat + vec);
}

void spmv(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
          hipStream_t s, int64_t seg) {
    FAMG_REQUIRE(m.spmv_ready(), AMG_ERR_UNSUPPORTED, "SpMV needs nnz < 2^31 (32-bit row pointers)");
    FAMG_REQUIRE(seg < (int64_t)m.seg_rows.size() - 1, AMG_ERR_INVALID, "SpMV segment out of range");
    FAMG_REQUIRE(mode != SPMV_SGS || epi.perm, AMG_ERR_INVALID, "SGS mode needs a permutation");
    if (g_launch_log) log_spmv(m, mode, epi, seg);
    Epi e{x, y, epi.b, epi.d, epi.perm, epi.dc, epi.dt, epi.dk};
    const dim3 block(256);
    if (m.gtx_on && (seg < 0 || m.rframe.on()) && gtx_supports(m, mode)) {
        spmv_gtx(m, x, y, mode, epi, s, seg);
        return;
    }
    if (m.gtc_on && (seg < 0 || m.rframe.on()) && gtc_supports(m, mode)) {
        spmv_gtc(m, x, y, mode, epi, s, seg);
        return;
    }
    FAMG_REQUIRE(mode != SPMV_SETDF || m.kernel == SPMV_KERNEL_SELLP || m.kernel == SPMV_KERNEL_BSR,
                 AMG_ERR_UNSUPPORTED, "SETDF needs a grid-transfer, pattern-SELL or 3x3-block restriction");
    if (m.kernel == SPMV_KERNEL_BSR) {
        FAMG_REQUIRE(mode != SPMV_SGS, AMG_ERR_UNSUPPORTED, "block storage has no SGS sweep");
        spmv_bsr(m, x, y, mode, epi, s, seg);
        return;
    }
    if (m.kernel == SPMV_KERNEL_SCS || (m.has_scs() && seg >= 0 && seg == m.scs_seg && mode != SPMV_SGS)) {
        FAMG_REQUIRE(mode != SPMV_SGS, AMG_ERR_UNSUPPORTED, "stencil-class storage has no SGS sweep");
        spmv_scs(m, x, y, mode, epi, s, seg);
        return;
    }
    if (m.kernel == SPMV_KERNEL_XS && seg < 0 && xs_supports(mode)) {  // other modes: CSR-stream below
        spmv_xs(m, x, y, mode, epi, s);
        return;
    }
    if (m.kernel == SPMV_KERNEL_SELLP) {
        FAMG_REQUIRE(mode != SPMV_SGS, AMG_ERR_UNSUPPORTED, "pattern SELL has no SGS sweep");
        spmv_sellp(m, x, y, mode, epi, s, seg);
        return;
    }
    if (mode == SPMV_SGS && m.has_dia() && m.dia_rowid) {  // color sweep of a color-permuted copy
        FAMG_REQUIRE(epi.perm == m.dia_rowid, AMG_ERR_INVALID, "SGS DIA: permutation mismatch");
        const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg];
        const int64_t r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
        if (r1 <= r0) return;
        DiaArgs a{};
        a.codes = m.dia_codes.get();
        a.ntab = (int32_t)m.dia_ntab;
        a.k = m.dia_k;
        a.row_begin = (int32_t)r0;
        a.row_end = (int32_t)r1;
        a.ncols = (int32_t)m.ncols;
        a.code_row0 = (int32_t)m.dia_r0;
        a.vtab = m.dia_vtab.get();
        for (int k = 0; k < m.dia_k; k++) a.off[k] = m.dia_off[k];
        a.e = e;
        const dim3 grid((unsigned)ceil_div(r1 - r0, 256));
        bool runs9 = m.dia_k == 27 && dia_runs();
        for (int j = 0; runs9 && j < 9; j++)
            runs9 = m.dia_off[3 * j + 1] == m.dia_off[3 * j] + 1 && m.dia_off[3 * j + 2] == m.dia_off[3 * j] + 2;
        if (runs9 && m.dia_vbits == 4 && m.dia_cw == 4) {
            spmv_dia_sgs_kernel<4, 4, 9><<<grid, block, 0, s>>>(a, m.dia_rowid);
            FAMG_CHECK_HIP(hipGetLastError());
            return;
        }
        if (runs9 && m.dia_vbits == 8 && m.dia_cw == 8) {
            spmv_dia_sgs_kernel<8, 8, 9><<<grid, block, 0, s>>>(a, m.dia_rowid);
            FAMG_CHECK_HIP(hipGetLastError());
            return;
        }
        switch (m.dia_vbits * 16 + m.dia_cw) {
        case 4 * 16 + 1: spmv_dia_sgs_kernel<4, 1><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 4 * 16 + 2: spmv_dia_sgs_kernel<4, 2><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 4 * 16 + 4: spmv_dia_sgs_kernel<4, 4><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 8 * 16 + 1: spmv_dia_sgs_kernel<8, 1><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 8 * 16 + 2: spmv_dia_sgs_kernel<8, 2><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 8 * 16 + 4: spmv_dia_sgs_kernel<8, 4><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        case 8 * 16 + 8: spmv_dia_sgs_kernel<8, 8><<<grid, block, 0, s>>>(a, m.dia_rowid); break;
        default: fail(AMG_ERR_INVALID, "SGS DIA: unsupported code layout");
        }
        FAMG_CHECK_HIP(hipGetLastError());
        return;
    }
    // a DIA row segment (the halo interior of a distributed level) runs DIA
    // even when the rest of the matrix is SELL storage
    if (m.kernel == SPMV_KERNEL_DIA ||
        (m.has_dia() && !m.dia_rowid && seg >= 0 && seg == m.dia_seg && mode != SPMV_SGS)) {
        FAMG_REQUIRE(mode != SPMV_SGS, AMG_ERR_UNSUPPORTED, "DIA storage has no SGS sweep");
        const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg];
        const int64_t r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
        if (r1 <= r0) return;
        DiaArgs a{};
        a.codes = m.dia_codes.get();
        a.ntab = (int32_t)m.dia_ntab;
        a.k = m.dia_k;
        a.row_begin = (int32_t)r0;
        a.row_end = (int32_t)r1;
        a.ncols = (int32_t)m.ncols;
        a.code_row0 = (int32_t)m.dia_r0;
        a.vtab = m.dia_vtab.get();
        for (int k = 0; k < m.dia_k; k++) a.off[k] = m.dia_off[k];
        a.e = e;
        a.band_bp = 0;
        {  // plane = the largest diagonal offset (a 3-D stencil's z neighbour)
            const int64_t plane = std::max<int64_t>(std::abs((int64_t)m.dia_off.front()), std::abs((int64_t)m.dia_off.back()));
            if (dia_bands() && plane % 4096 == 0 && plane >= 8 * 4096 && (r1 - r0) % plane == 0)
                a.band_bp = (int32_t)(plane / 512);
        }
        const dim3 grid((unsigned)ceil_div(r1 - r0, 512));
        const int key = m.dia_vbits * 16 + m.dia_cw;
        const bool nt = dia_nt();
        // 27 diagonals in nine runs of three consecutive offsets (27-point
        // stencil), or the 7-point pattern with its x run in the middle
        bool runs9 = m.dia_k == 27 && dia_runs();
        for (int j = 0; runs9 && j < 9; j++)
            runs9 = m.dia_off[3 * j + 1] == m.dia_off[3 * j] + 1 && m.dia_off[3 * j + 2] == m.dia_off[3 * j] + 2;
        const bool run7 = dia_run7(m);
        const bool dk = dia_dk(m, epi);
        const int runs9i = runs9 ? 9 : run7 ? -1 : 0;
        const int pat = m.dia_pat ? m.dia_pat : runs9 && dia_pat27() && (key == 4 * 16 + 4 || key == 8 * 16 + 8) ? 27 : 0;
        if (pat) {
        const bool cst = pat == 27 && m.dia_cst && seg < 0 && dia_cst_enabled();
        if (cst) {
            a.gnx = m.dia_cst_n[0];
            a.gny = m.dia_cst_n[1];
            a.gnz = m.dia_cst_n[2];
            for (int k = 0; k < 27; k++) a.cst[k] = m.dia_cst_v[k];
        }
#define FAMG_DIAP2(M, VB, CW, P)                                                                  \
    if (cst) spmv_dia_pat_kernel<M, VB, CW, P, (P == 27)><<<grid, block, 0, s>>>(a);              \
    else spmv_dia_pat_kernel<M, VB, CW, P><<<grid, block, 0, s>>>(a);
#define FAMG_DIAP(VB, CW, P)                                                                        \
    switch (mode) {                                                                               \
    case SPMV_SET: FAMG_DIAP2(SPMV_SET, VB, CW, P) break;                                            \
    case SPMV_ADD: FAMG_DIAP2(SPMV_ADD, VB, CW, P) break;                                            \
    case SPMV_RESID: FAMG_DIAP2(SPMV_RESID, VB, CW, P) break;                                        \
    case SPMV_JACOBI:                                                                             \
        if (e.dc) {                                                                               \
            FAMG_DIAP2(DIA_JACOBI_DC, VB, CW, P)                                                     \
        } else {                                                                                  \
            FAMG_DIAP2(SPMV_JACOBI, VB, CW, P)                                                       \
        }                                                                                         \
        break;                                                                                    \
    case SPMV_RESID0: FAMG_DIAP2(SPMV_RESID0, VB, CW, P) break;                                      \
    case SPMV_ADD0: FAMG_DIAP2(SPMV_ADD0, VB, CW, P) break;                                          \
    default: break;                                                                               \
    }
            FAMG_REQUIRE(pat == 33 || pat == 27, AMG_ERR_INVALID, "DIA: unsupported run pattern");
            if (pat == 33 && key == 8 * 16 + 9) {
                FAMG_DIAP(8, 9, 33)
            } else if (pat == 33 && key == 4 * 16 + 5) {
                FAMG_DIAP(4, 5, 33)
            } else if (pat == 27 && key == 8 * 16 + 8) {
                FAMG_DIAP(8, 8, 27)
            } else if (pat == 27 && key == 4 * 16 + 4) {
                FAMG_DIAP(4, 4, 27)
            } else {
                fail(AMG_ERR_INVALID, "DIA: unsupported code layout");
            }
#undef FAMG_DIAP
#undef FAMG_DIAP2
            FAMG_CHECK_HIP(hipGetLastError());
            return;
        }
        const bool cst7 = runs9i == -1 && m.dia_cst && m.dia_k == 7 && seg < 0 && dia_cst_enabled();
        if (cst7) {
            a.gnx = m.dia_cst_n[0];
            a.gny = m.dia_cst_n[1];
            a.gnz = m.dia_cst_n[2];
            for (int k = 0; k < 7; k++) a.cst[k] = m.dia_cst_v[k];
        }
#define FAMG_DIA2(M, VB, CW) launch_dia<M, VB, CW>(runs9i, nt, grid, block, s, a, cst7);
#define FAMG_DIA(VB, CW)                                                                          \
    switch (mode) {                                                                               \
    case SPMV_SET: FAMG_DIA2(SPMV_SET, VB, CW) break;                                             \
    case SPMV_ADD: FAMG_DIA2(SPMV_ADD, VB, CW) break;                                             \
    case SPMV_RESID: FAMG_DIA2(SPMV_RESID, VB, CW) break;                                         \
    case SPMV_JACOBI:                                                                             \
        if (dk) {                                                                                 \
            FAMG_DIA2(DIA_JACOBI_DK, VB, CW)                                                      \
        } else if (e.dc) {                                                                        \
            FAMG_DIA2(DIA_JACOBI_DC, VB, CW)                                                      \
        } else {                                                                                  \
            FAMG_DIA2(SPMV_JACOBI, VB, CW)                                                        \
        }                                                                                         \
        break;                                                                                    \
    case SPMV_RESID0:                                                                             \
        if (dk) {                                                                                 \
            FAMG_DIA2(DIA_RESID0_DK, VB, CW)                                                      \
        } else if (e.dc && dia_rc_enabled()) {                                                    \
            FAMG_DIA2(DIA_RESID0_DC, VB, CW)                                                      \
        } else {                                                                                  \
            FAMG_DIA2(SPMV_RESID0, VB, CW)                                                        \
        }                                                                                         \
        break;                                                                                    \
    case SPMV_ADD0: FAMG_DIA2(SPMV_ADD0, VB, CW) break;                                           \
    default: break;                                                                               \
    }
        switch (key) {
        case 4 * 16 + 1: FAMG_DIA(4, 1) break;
        case 4 * 16 + 2: FAMG_DIA(4, 2) break;
        case 4 * 16 + 4: FAMG_DIA(4, 4) break;
        case 8 * 16 + 1: FAMG_DIA(8, 1) break;
        case 8 * 16 + 2: FAMG_DIA(8, 2) break;
        case 8 * 16 + 4: FAMG_DIA(8, 4) break;
        case 8 * 16 + 8: FAMG_DIA(8, 8) break;
        default: fail(AMG_ERR_INVALID, "DIA: unsupported code layout");
        }
#undef FAMG_DIA
#undef FAMG_DIA2
    } else if (m.kernel == SPMV_KERNEL_SELL) {
        const int64_t s0 = seg < 0 ? 0 : m.seg_slc[seg];
        const int64_t s1 = seg < 0 ? m.nslices : m.seg_slc[seg + 1];
        if (s1 <= s0) return;
        SellArgs a{m.sell_row0.get(), m.sell_soff.get(), m.sell_desc.get(), m.sell_base.get(),
                   m.sell_data.get(), (int32_t)s0, (int32_t)(s1 - s0), e, m.sell_vtab.get(),
                   (int32_t)m.sell_ntab, 1};
        // value codes: two slices per wave when there are enough waves to fill the chip twice over
        const int lay = m.sell_vbits ? 4 : 0;
        if (sell_slices_per_wave(lay, mode) == 2 && s1 - s0 >= SELL_PAIR_MIN_SLICES) a.spw = 2;
        const dim3 grid((unsigned)ceil_div(s1 - s0, 4 * a.spw * sell_groups_per_wave(lay)));
        if (m.sell_short && seg < 0 && mode != SPMV_SGS && mode != SPMV_RESID0 && sell_short_enabled()) {
            const dim3 g2((unsigned)ceil_div(s1 - s0, 8));
            if (m.sell_vbits == 4) {
                FAMG_LAUNCH_MODES(spmv_sell_short_kernel, g2, block, s, a, FAMG_LAY4)
            } else if (m.sell_vbits == 8) {
                FAMG_LAUNCH_MODES(spmv_sell_short_kernel, g2, block, s, a, FAMG_LAY8)
            } else {
                FAMG_LAUNCH_MODES(spmv_sell_short_kernel, g2, block, s, a, FAMG_LAY16)
            }
        } else if (m.sell_vbits == 4) {
            FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a, FAMG_LAY4)
        } else if (m.sell_vbits == 8) {
            FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a, FAMG_LAY8)
        } else if (m.sell_vbits == 16 && m.sell_ntab <= 8192 && mode != SPMV_SGS &&
                   ((sell_t16_mode() < 0 && m.nnz >= 32 * m.nrows) || sell_t16_mode() > 0)) {
            const int nvb = (int)grid.x;
            const dim3 g2((unsigned)(sell_t16_mode() > 0 ? std::min(nvb, 256 * sell_t16_mode()) : nvb));
            const size_t lds = (size_t)m.sell_ntab * sizeof(double);
            switch (mode) {
            case SPMV_SET: spmv_sell_t16_kernel<SPMV_SET><<<g2, block, lds, s>>>(a, nvb); break;
            case SPMV_ADD: spmv_sell_t16_kernel<SPMV_ADD><<<g2, block, lds, s>>>(a, nvb); break;
            case SPMV_RESID: spmv_sell_t16_kernel<SPMV_RESID><<<g2, block, lds, s>>>(a, nvb); break;
            case SPMV_JACOBI: spmv_sell_t16_kernel<SPMV_JACOBI><<<g2, block, lds, s>>>(a, nvb); break;
            case SPMV_RESID0: spmv_sell_t16_kernel<SPMV_RESID0><<<g2, block, lds, s>>>(a, nvb); break;
            case SPMV_ADD0: spmv_sell_t16_kernel<SPMV_ADD0><<<g2, block, lds, s>>>(a, nvb); break;
            default: break;
            }
        } else if (m.sell_vbits == 16) {
            FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a, FAMG_LAY16)
        } else if (m.sell_paired) {
            FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a, FAMG_LAY1)
        } else {
            FAMG_LAUNCH_MODES(spmv_sell_kernel, grid, block, s, a, FAMG_LAY0)
        }
    } else if (m.kernel == SPMV_KERNEL_VECTOR) {
        const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg];
        const int64_t r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
        if (r1 <= r0) return;
        VecArgs a{m.rp32.get(), m.col.get(), m.vec_off.get(), m.val.get(), m.vec_codes.get(), m.sell_vtab.get(),
                  (int32_t)r0, (int32_t)(r1 - r0), e};
        const int wpr = flag(FLAG_VEC_WPR) ? (int)flag(FLAG_VEC_WPR) : m.vec_wpr;
        const dim3 grid((unsigned)ceil_div(r1 - r0, 4 / wpr));
        const int key = m.vec_vbits * 2 + (m.vec_o16 ? 1 : 0);
#define FAMG_VECW(W)                                                                                   \
        switch (key) {                                                                                 \
        case 0: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(0, false, W)) break;  \
        case 1: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(0, true, W)) break;   \
        case 16: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(8, false, W)) break; \
        case 17: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(8, true, W)) break;  \
        case 32: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(16, false, W)) break;\
        default: FAMG_LAUNCH_MODES(spmv_vector_kernel, grid, block, s, a, FAMG_VEC(16, true, W)) break; \
        }
        if (wpr == 4) { FAMG_VECW(4) }
        else if (wpr == 2) { FAMG_VECW(2) }
        else { FAMG_VECW(1) }
#undef FAMG_VECW
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
