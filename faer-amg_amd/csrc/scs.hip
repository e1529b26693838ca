// scs.hip -- stencil-class storage for structured Galerkin operators.
//
// The coarse operators of a box-aggregation hierarchy on a structured grid are
// stencils whose rows repeat bit for bit away from the boundary: A_1 of the
// 256^3 cycle (2M rows, 32 entries per row) has 125 distinct rows up to a shift
// (5^3 boundary-distance classes), A_2 (262K rows, 168 entries) 2197 (13^3).  The
// storage keeps
//   offs[K]      the sorted union of all rows' column offsets (col - row), K
//                padded to a multiple of 8 with offset 0,
//   dict[C][K]   for every class c its value at every offset (+0.0 where the
//                class has no entry), class-major: a wave meets a handful of
//                classes (rows along a grid line differ only near its ends), so
//                an XCD touches only the stencils of its rows' classes,
//   cls[n]       one 8/16-bit class id per row,
// i.e. 1-2 B per row instead of 1-8 B per entry.  Row i's sum walks the K
// offsets in ascending order with fma -- the stored entries in ascending column
// order with exact zero terms between them, which is the oracle's CSR order:
// row sums bitwise equal (x finite).  Offsets leaving [0, n) carry +0.0 and are
// clamped.  Built with 64 <= K <= 1024, <= 65536 classes, a dictionary of <= 16
// MiB and at most half the bytes of the storage finalize chose, for a square
// matrix or for the halo-interior row segment of a distributed level (rows that
// read owned columns only; the boundary segments keep SELL-64).
#include <algorithm>
#include <type_traits>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "famg.hpp"
#include "tuning.hpp"

namespace famg {

constexpr int SCS_KMAX = 1024;
constexpr int SCS_KMIN = 64;
constexpr int SCS_U = 8;  // offsets per load group (K is padded to a multiple)

struct ScsArgs {
    const void *cls;
    const double *dict;
    const int32_t *offs;
    int32_t k, nclass, row_begin, row_end, ncols;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
};

typedef double scs_dbl2_t __attribute__((ext_vector_type(2), aligned(8)));
typedef double scs_dbl2a_t __attribute__((ext_vector_type(2)));

// x operands of rows (r, r+1) at column c = r + off: one 16-B load at clamp(c, 0,
// ncols - 2) and selects (a column outside [0, ncols) belongs to a +0.0 term, so
// any finite value will do there)
template <int MODE>
__device__ __forceinline__ void scs_x2(const ScsArgs &a, int c, double &xa, double &xb) {
    const int p = min(max(c, 0), a.ncols - 2);
    scs_dbl2_t v = *reinterpret_cast<const scs_dbl2_t *>(a.x + p);
    xa = c > p ? v.y : v.x;
    xb = c < p ? v.x : v.y;
}

// Two adjacent rows per lane (16-B x loads); the dictionary is read through
// the caches (staging A_1's 40 KB dictionary in LDS per workgroup measured the
// same, 47 vs 48 us).
template <int MODE, int IB>
__global__ __launch_bounds__(256) void spmv_scs_kernel(ScsArgs a) {
    const double *dict = a.dict;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int row = a.row_begin + 2 * (blk * 256 + (int)threadIdx.x);
    const bool l0 = row < a.row_end, l1 = row + 1 < a.row_end;
    const int r0 = l0 ? row : a.row_begin;
    auto cls_of = [&](int r) {
        return IB == 1 ? (int)static_cast<const uint8_t *>(a.cls)[r] : (int)static_cast<const uint16_t *>(a.cls)[r];
    };
    const int c0 = cls_of(r0), c1 = l1 ? cls_of(row + 1) : c0;
    double br[2] = {0.0, 0.0}, xr[2] = {0.0, 0.0}, dr[2] = {0.0, 0.0}, yr[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 2; j++) {  // epilogue operands first
        if (!(j ? l1 : l0)) continue;
        const int i = row + j;
        if constexpr (MODE == SPMV_RESID) br[j] = a.b[i];
        if constexpr (MODE == SPMV_ADD) yr[j] = a.y[i];
        if constexpr (MODE == SPMV_JACOBI) {
            xr[j] = a.x[i];
            br[j] = a.b[i];
            dr[j] = a.dc ? a.dt[a.dc[i]] : a.d[i];
        }
    }
    const double *da = dict + (int64_t)c0 * a.k, *db = dict + (int64_t)c1 * a.k;
    double acc0 = 0.0, acc1 = 0.0;
    for (int k0 = 0; k0 < a.k; k0 += SCS_U) {
        double va[SCS_U], vb[SCS_U], xa[SCS_U], xb[SCS_U];
#pragma unroll
        for (int u = 0; u < SCS_U; u++) scs_x2<MODE>(a, r0 + a.offs[k0 + u], xa[u], xb[u]);
        // dictionary values of offsets (k, k+1) as one 16-B load (rows of K = 8j doubles)
#pragma unroll
        for (int u = 0; u < SCS_U; u += 2) {
            const scs_dbl2a_t pa = *reinterpret_cast<const scs_dbl2a_t *>(da + k0 + u);
            const scs_dbl2a_t pb = *reinterpret_cast<const scs_dbl2a_t *>(db + k0 + u);
            va[u] = pa.x;
            va[u + 1] = pa.y;
            vb[u] = pb.x;
            vb[u + 1] = pb.y;
        }
#pragma unroll
        for (int u = 0; u < SCS_U; u++) {
            acc0 = fma(va[u], xa[u], acc0);
            acc1 = fma(vb[u], xb[u], acc1);
        }
    }
    const double acc[2] = {acc0, acc1};
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (!(j ? l1 : l0)) continue;
        const int i = row + j;
        if constexpr (MODE == SPMV_SET) a.y[i] = acc[j];
        else if constexpr (MODE == SPMV_ADD) a.y[i] = yr[j] + acc[j];
        else if constexpr (MODE == SPMV_RESID) a.y[i] = br[j] - acc[j];
        else a.y[i] = xr[j] + dr[j] * (br[j] - acc[j]);  // JACOBI
    }
}

// Few long rows (A_3 of the 256^3 cycle: 32768 rows of 638 entries, 15625
// classes -- nearly every row its own): one row per wave, lane q takes the
// offset pairs 2q, 2q + 1 of every 128-offset block (16-B dictionary and 8-B
// offset loads, both coalesced), then a fixed butterfly -- deterministic;
// rounding-level differences from the oracle's sequential order, covered by
// the V-cycle tolerance.  Two dependent round trips per row: the class id and
// ALL the row's offsets first (the offsets do not depend on the class), then
// the dictionary row and every x operand at once.
template <int MODE, int IB>
__global__ __launch_bounds__(256) void spmv_scs_lanes_kernel(ScsArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int row = a.row_begin + __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    if (row >= a.row_end) return;
    const int lane = threadIdx.x & 63;
    const int c = IB == 1 ? (int)static_cast<const uint8_t *>(a.cls)[row] : (int)static_cast<const uint16_t *>(a.cls)[row];
    constexpr int NB = SCS_KMAX / 128;  // 128-offset blocks (K <= 1024, a multiple of 8)
    const int nb = (a.k + 127) >> 7;
    int2 of[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const int kk = 128 * j + 2 * lane;
        of[j] = (j < nb && kk < a.k) ? *reinterpret_cast<const int2 *>(a.offs + kk) : int2{0, 0};
    }
    double br = 0.0, xr = 0.0, dr = 0.0, yr = 0.0;
    if (lane == 0) {  // epilogue operands
        if constexpr (MODE == SPMV_RESID) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
        if constexpr (MODE == SPMV_JACOBI) {
            xr = a.x[row];
            br = a.b[row];
            dr = a.dc ? a.dt[a.dc[row]] : a.d[row];
        }
    }
    double x0[NB], x1[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        if (j < nb) {
            x0[j] = a.x[min(max(row + of[j].x, 0), a.ncols - 1)];
            x1[j] = a.x[min(max(row + of[j].y, 0), a.ncols - 1)];
        }
    }
    const double *dct = a.dict + (int64_t)c * a.k;
    scs_dbl2a_t v[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const int kk = 128 * j + 2 * lane;
        if (j < nb) v[j] = kk < a.k ? *reinterpret_cast<const scs_dbl2a_t *>(dct + kk) : scs_dbl2a_t{0.0, 0.0};
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        if (j < nb) {
            acc = fma(v[j].x, x0[j], acc);
            acc = fma(v[j].y, x1[j], acc);
        }
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    if (lane == 0) {
        if constexpr (MODE == SPMV_SET) a.y[row] = acc;
        else if constexpr (MODE == SPMV_ADD) a.y[row] = yr + acc;
        else if constexpr (MODE == SPMV_RESID) a.y[row] = br - acc;
        else a.y[row] = xr + dr * (br - acc);  // JACOBI
    }
}

// x-staged stencil classes on a 3-D grid (the rows are the points of an
// nx x ny x nz grid, x fastest, and every nonzero's offset maps to a grid
// neighbour within radii rx, ry, rz).  One workgroup per tile of tx x ty x tz
// points: it stages the tile's x window -- the tile plus the halo, 0.0 outside
// the grid -- in LDS (one read of each x value from L2/HBM per window instead of
// one cache gather per entry), then each lane walks the K offsets of its RL rows
// in ascending order reading x from LDS at its window position + lo[k].  A
// wave whose rows share a class (interior tiles) reads the dictionary through
// scalar loads.  Arithmetic is spmv_scs_kernel's: fma over the K offsets in
// ascending order, absent entries +0.0 times a finite value (an x entry or the
// halo's 0.0), so the row sums are bitwise the oracle's CSR sums.
struct XscsArgs {
    const void *cls;
    const double *dict;
    const int32_t *lo;
    int32_t k, kr;  // offsets per dictionary row (a multiple of 8) / before the padding
    int nx, ny, nz, tx, ty, tz, rx, ry, rz, wx, wy, wz, ntx, nty;
    int ws;  // LDS row stride of the window (>= wx)
    // staged planes: local plane z is loadable for zlo <= z < zhi (else 0.0) and
    // starts at z * plane + (z < 0 ? add_lo : z >= nz ? add_hi : 0) -- a rank-local
    // matrix's ghost planes (SlabFrame); single GPU: 0, nz, 0, 0
    int zlo, zhi, tile0;
    int64_t add_lo, add_hi;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
    // float reciprocals of wx, wy, tx, ty: q / d as (int)((q + 0.5f) * r), exact for
    // the q < 2^14, d <= 128 used here (checked on the host for every q of a launch);
    // the runtime integer divisions of the staging loop were the kernel's largest
    // VALU cost (PMC, profiles/r04/pmc_xscs_summary.json)
    float rwx, rwy, rtx, rty;
};

template <int MODE, int IB, int RL>
__global__ __launch_bounds__(256) void spmv_xscs_kernel(XscsArgs a) {
    extern __shared__ double win[];
    const int tid = threadIdx.x;
    const int t = a.tile0 + xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int x0 = tix * a.tx, y0 = tiy * a.ty, z0 = tiz * a.tz;
    const int T = a.tx * a.ty * a.tz;
    const int64_t plane = (int64_t)a.nx * a.ny;
    auto cls_of = [&](int64_t r) {
        return IB == 1 ? (int)static_cast<const uint8_t *>(a.cls)[r] : (int)static_cast<const uint16_t *>(a.cls)[r];
    };
    // the rows' class ids and epilogue operands first: their loads overlap the staging
    int wb[RL], c[RL];
    int64_t gi[RL];
    bool live[RL];
    double br[RL], xr[RL], dr[RL], yr[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) {
        const int lt = tid + 256 * j;
        const int lq = fdiv_rcp(lt, a.rtx), lz = fdiv_rcp(lq, a.rty);
        const int lx = lt - lq * a.tx, ly = lq - lz * a.ty;
        const int gx = x0 + lx, gy = y0 + ly, gz = z0 + lz;
        live[j] = lt < T && gx < a.nx && gy < a.ny && gz < a.nz;
        gi[j] = live[j] ? (int64_t)gz * plane + (int64_t)gy * a.nx + gx
                        : (int64_t)z0 * plane + (int64_t)y0 * a.nx + x0;  // the tile's first point
        wb[j] = live[j] ? ((lz + a.rz) * a.wy + ly + a.ry) * a.ws + lx + a.rx
                        : (a.rz * a.wy + a.ry) * a.ws + a.rx;
        c[j] = cls_of(gi[j]);
        br[j] = xr[j] = dr[j] = yr[j] = 0.0;
        if (live[j]) {
            if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) br[j] = a.b[gi[j]];
            if constexpr (MODE == SPMV_ADD) yr[j] = a.y[gi[j]];
            if constexpr (MODE == SPMV_JACOBI) {  // (x at the row itself: from the staged window below)
                br[j] = a.b[gi[j]];
                dr[j] = a.dc ? a.dt[a.dc[gi[j]]] : a.d[gi[j]];
            }
        }
    }
    // stage the window: rows of wx consecutive x values, 0.0 outside the grid.
    // RESID0 (the zero-guess step folded into the residual): the staged operand
    // is the iterate d*x that vec_mul(_coded) would have stored, so the sums are
    // the unfolded residual's bitwise
    const int W = a.wx * a.wy * a.wz;
    constexpr int PF = 8;
    for (int p0 = tid; p0 < W; p0 += 256 * PF) {
        double v[PF];
        int si[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int p = p0 + 256 * u;
            const int q = fdiv_rcp(p, a.rwx), pz = fdiv_rcp(q, a.rwy);
            const int px = p - q * a.wx, py = q - pz * a.wy;
            si[u] = q * a.ws + px;  // (pz wy + py) ws + px
            const int gx = x0 - a.rx + px, gy = y0 - a.ry + py, gz = z0 - a.rz + pz;
            const bool in = p < W && (unsigned)gx < (unsigned)a.nx && (unsigned)gy < (unsigned)a.ny && gz >= a.zlo &&
                            gz < a.zhi;
            const int64_t g = (int64_t)gz * plane + (gz < 0 ? a.add_lo : gz >= a.nz ? a.add_hi : 0) +
                              (int64_t)gy * a.nx + gx;
            if constexpr (MODE == SPMV_RESID0) v[u] = in ? (a.dc ? a.dt[a.dc[g]] : a.d[g]) * a.x[g] : 0.0;
            else v[u] = in ? a.x[g] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < PF; u++)
            if (p0 + 256 * u < W) win[si[u]] = v[u];
    }
    __syncthreads();
    if constexpr (MODE == SPMV_JACOBI) {
#pragma unroll
        for (int j = 0; j < RL; j++) xr[j] = win[wb[j]];  // the staged x_i (the window holds x itself)
    }
    bool uni = true;
    int cu[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) {
        cu[j] = __builtin_amdgcn_readfirstlane(c[j]);
        uni = uni && __all(c[j] == cu[j]);
    }
    double acc[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) acc[j] = 0.0;
    if (uni) {  // wave-uniform classes: dictionary values through scalar loads
        // groups of UG offsets: scalar and LDS loads share the lgkm counter, so
        // each group is one wait for its offsets and values and one for its reads
        // (16 per group on one-row-per-lane tiles: C2 A_3 JACOBI 35.6 -> 31.8 us,
        // the other levels within 1 us)
        auto group = [&](auto ug, int k0) {
            constexpr int UG = decltype(ug)::value;
            int l[UG];
#pragma unroll
            for (int u = 0; u < UG; u++) l[u] = a.lo[k0 + u];
            double xv[RL][UG], v[RL][UG];
#pragma unroll
            for (int j = 0; j < RL; j++)
#pragma unroll
                for (int u = 0; u < UG; u++) {
                    xv[j][u] = win[wb[j] + l[u]];
                    v[j][u] = a.dict[(int64_t)cu[j] * a.k + k0 + u];
                }
#pragma unroll
            for (int j = 0; j < RL; j++)
#pragma unroll
                for (int u = 0; u < UG; u++) acc[j] = fma(v[j][u], xv[j][u], acc[j]);
        };
        // the padding offsets (+0.0 at the row itself) are skipped: adding +0.0 x
        // to a sum that started at +0.0 never changes it
        int k0 = 0;
        if (RL == 1)
            for (; k0 + 16 <= a.kr; k0 += 16) group(std::integral_constant<int, 16>{}, k0);
        for (; k0 + SCS_U <= a.kr; k0 += SCS_U) group(std::integral_constant<int, SCS_U>{}, k0);
        for (; k0 < a.kr; k0++) group(std::integral_constant<int, 1>{}, k0);
    } else {
        for (int k0 = 0; k0 < a.k; k0 += SCS_U) {
            int l[SCS_U];
#pragma unroll
            for (int u = 0; u < SCS_U; u++) l[u] = a.lo[k0 + u];
            double xv[RL][SCS_U], v[RL][SCS_U];
#pragma unroll
            for (int j = 0; j < RL; j++) {
                const double *dj = a.dict + (int64_t)c[j] * a.k + k0;
#pragma unroll
                for (int u = 0; u < SCS_U; u += 2) {
                    const scs_dbl2a_t pv = *reinterpret_cast<const scs_dbl2a_t *>(dj + u);
                    v[j][u] = pv.x;
                    v[j][u + 1] = pv.y;
                }
#pragma unroll
                for (int u = 0; u < SCS_U; u++) xv[j][u] = win[wb[j] + l[u]];
            }
#pragma unroll
            for (int j = 0; j < RL; j++)
#pragma unroll
                for (int u = 0; u < SCS_U; u++) acc[j] = fma(v[j][u], xv[j][u], acc[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < RL; j++) {
        if (!live[j]) continue;
        const int64_t i = gi[j];
        if constexpr (MODE == SPMV_SET) a.y[i] = acc[j];
        else if constexpr (MODE == SPMV_ADD) a.y[i] = yr[j] + acc[j];
        else if constexpr (MODE == SPMV_RESID || MODE == SPMV_RESID0) a.y[i] = br[j] - acc[j];
        else a.y[i] = xr[j] + dr[j] * (br[j] - acc[j]);  // JACOBI
    }
}

// the lanes-per-row kernel for row ranges of < SCS_LANES_ROWS rows with >= 256
// offsets (A/B switch FAMG_SCS_LANES=0: no stencil classes for them)
constexpr int64_t SCS_LANES_ROWS = 131072;
static bool scs_lanes_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_SCS_LANES");
        return !(e && e[0] == '0');
    }();
    return on;
}

static bool scs_rows_pref() {
    static const bool on = [] {
        const char *e = getenv("FAMG_SCS_ROWS");
        return e && e[0] == '1';
    }();
    return on;
}

static bool scs_disabled() {
    static const bool off = [] {
        const char *e = getenv("FAMG_NO_SCS");
        return e && e[0] == '1';
    }();
    return off;
}

void scs_release(GpuCsr &m) {
    m.scs_cls.release();
    m.scs_dict.release();
    m.scs_offs.release();
    m.scs_k = m.scs_nclass = m.scs_ib = 0;
    m.scs_kr = 0;
    m.scs_seg = -1;
    m.scs_lanes = false;
    m.xscs = false;
    m.xscs_tile_src = 0;
    m.xscs_lo.release();
}

// A/B switch FAMG_XSCS=0: no x-staged stencil classes; FAMG_XSCS_TILE=tx,ty,tz
// forces the tile
static bool xscs_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_XSCS");
        return !(e && e[0] == '0');
    }();
    return on;
}

// The grid hint applies to the whole square matrix.
static bool grid_applies(const GpuCsr &m) {
    return xscs_enabled() && m.grid[0] > 0 && m.grid[1] > 0 && m.grid[2] > 0 && m.nrows == m.ncols &&
           m.grid[0] * m.grid[1] * m.grid[2] == m.nrows && m.nrows < (int64_t(1) << 31);
}

// Tile t for m's x-staged kernel: the window offset of every stencil offset,
// relative to the row's own window position.
// The window's LDS row stride for tile t: the stride in [wx, wx + 31] (window
// <= 64 KB) whose first wave's ds_read_b64 lanes meet the fewest bank repeats
// (lanes 0-31 and 32-63 each serviced together, bank = dword mod 64,
// MI355X_MICROARCH.md LDS table); every stencil offset shifts all lanes alike,
// so the row positions decide.  A_1 of the 7-point cycle on 8 x 8 x 8 tiles:
// stride 12 put rows y and y + 3 on the same banks (PMC: 45 % of the LDS cycles
// were bank conflicts).
static int xscs_stride(const int *t, int wx, int wy, int wz) {
    int best = wx, best_cost = 1 << 30;
    for (int s = wx; s < wx + 32 && (int64_t)s * wy * wz * 8 <= 64 * 1024; s++) {
        int cost = 0;
        for (int g = 0; g < 2; g++) {
            int cnt[64] = {0};
            for (int lane = 32 * g; lane < 32 * g + 32; lane++) {
                const int lx = lane % t[0], ly = (lane / t[0]) % t[1], lz = lane / (t[0] * t[1]);
                const int a = (lz * wy + ly) * s + lx;
                cnt[(2 * a) & 63]++;
                cnt[(2 * a + 1) & 63]++;
            }
            cost += *std::max_element(cnt, cnt + 64);
        }
        if (cost < best_cost) {
            best_cost = cost;
            best = s;
        }
    }
    return best;
}

static void xscs_set_tile(GpuCsr &m, const int *t) {
    const int rx = m.xscs_r[0], ry = m.xscs_r[1], rz = m.xscs_r[2];
    const int wx = t[0] + 2 * rx, wy = t[1] + 2 * ry;
    const int ws = xscs_stride(t, wx, wy, t[2] + 2 * rz);
    const int Kp = (int)(m.xscs_steps.size() / 3);
    std::vector<int32_t> lo(Kp);
    for (int k = 0; k < Kp; k++)
        lo[k] = (m.xscs_steps[3 * k + 2] * wy + m.xscs_steps[3 * k + 1]) * ws + m.xscs_steps[3 * k];
    m.xscs_ws = ws;
    m.xscs_lo.resize(Kp);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.xscs_lo.get(), lo.data(), Kp * 4, hipMemcpyHostToDevice, m.ctx->stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(m.ctx->stream));
    for (int q = 0; q < 3; q++) m.xscs_t[q] = t[q];
    // the staging loops divide by the window and tile extents through float
    // reciprocals: checked once here, at storage build, not per launch
    const int wz = t[2] + 2 * rz;
    m.xscs_fdiv = fdiv_exact(wx * wy * wz, wx, 1.0f / (float)wx) && fdiv_exact(wy * wz, wy, 1.0f / (float)wy) &&
                  fdiv_exact(1024, t[0], 1.0f / (float)t[0]) && fdiv_exact(1024 / t[0] + 1, t[1], 1.0f / (float)t[1]);
}

// Decompose the offsets into grid steps (dx, dy, dz) (centred residues), check
// that every nonzero entry's step stays inside the grid, pick the tile and store
// the window offsets: m.xscs on success.
static bool xscs_setup(GpuCsr &m, const std::vector<int32_t> &offs, int Kp, const std::vector<int64_t> &rp,
                       const std::vector<int32_t> &col, const std::vector<double> &val) {
    const int64_t nx = m.grid[0], ny = m.grid[1], nz = m.grid[2], pl = nx * ny, n = m.nrows;
    const int K = (int)offs.size();
    std::vector<int> dx(K), dy(K), dz(K);
    int rx = 0, ry = 0, rz = 0;
    for (int k = 0; k < K; k++) {
        const int64_t o = offs[k];
        int64_t ex = ((o % nx) + nx) % nx;
        if (ex > nx / 2) ex -= nx;
        const int64_t q = (o - ex) / nx;
        int64_t ey = ((q % ny) + ny) % ny;
        if (ey > ny / 2) ey -= ny;
        const int64_t ez = (q - ey) / ny;
        dx[k] = (int)ex;
        dy[k] = (int)ey;
        dz[k] = (int)ez;
        rx = std::max(rx, std::abs(dx[k]));
        ry = std::max(ry, std::abs(dy[k]));
        rz = std::max<int>(rz, (int)std::min<int64_t>(std::abs(ez), INT32_MAX / 4));
    }
    if (rx > 16 || ry > 16 || rz > 16) return false;
    // planes a nonzero may reach: the grid, or a rank-local matrix's owned + ghost planes
    const int64_t zlo = m.cframe.on() ? -m.cframe.gl : 0, zhi = m.cframe.on() ? nz + m.cframe.gh : nz;
    bool ok = true;
#pragma omp parallel for schedule(static) reduction(&& : ok)
    for (int64_t i = 0; i < n; i++) {
        const int64_t x = i % nx, y = (i / nx) % ny, z = i / pl;
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            if (val[e] == 0.0) continue;
            const int32_t o = (int32_t)((int64_t)col[e] - i);
            const int k = (int)(std::lower_bound(offs.begin(), offs.end(), o) - offs.begin());
            const int64_t X = x + dx[k], Y = y + dy[k], Z = z + dz[k];
            if (X < 0 || X >= nx || Y < 0 || Y >= ny || Z < zlo || Z >= zhi) ok = false;
        }
    }
    if (!ok) return false;
    // tile: smallest modelled time -- per CU, ds_read_b64 at 2 clk per wave and
    // offset plus the window staged at ~64 B/clk, in rounds of 256 workgroups,
    // plus a latency per round of resident workgroups
    int best[3] = {0, 0, 0};
    double best_cost = 1e300;
    auto cands = [](int64_t ext, bool z) {
        std::vector<int> c;
        for (int t : {1, 2, 4, 8, 16, 32, 64})
            if ((z || t >= 4) && t <= ext) c.push_back(t);
        if (ext < 64 && (c.empty() || c.back() != ext)) c.push_back((int)ext);
        return c;
    };
    for (int tx : cands(nx, false))
        for (int ty : cands(ny, false))
            for (int tz : cands(nz, true)) {
                const int64_t T = (int64_t)tx * ty * tz;
                const int64_t W = (int64_t)(tx + 2 * rx) * (ty + 2 * ry) * (tz + 2 * rz);
                if (T > 1024 || T < std::min<int64_t>(64, n) || W * 8 > 64 * 1024) continue;
                // one row per lane wherever the grid gives >= 1024 such tiles: the
                // walk is latency-bound, so resident waves matter more than halo
                // bytes (A_2 of the 256^3 cycle: 1024-row tiles, one wave per SIMD,
                // ran 51 us against 40 on the cache-gathering kernel)
                if (T > 256 && n >= 1024 * 256) continue;
                const int64_t ntiles = ceil_div(nx, tx) * ceil_div(ny, ty) * ceil_div(nz, tz);
                const double occ = std::min(4.0, std::floor(160.0 * 1024 / (W * 8.0)));
                const double rounds = std::ceil(ntiles / 256.0);
                const double cost = rounds * ((double)std::max<int64_t>(T, 64) * Kp / 32.0 + W / 8.0) +
                                    1500.0 * std::ceil(ntiles / (256.0 * occ));
                if (cost < best_cost) {
                    best_cost = cost;
                    best[0] = tx; best[1] = ty; best[2] = tz;
                }
            }
    if (const char *e = getenv("FAMG_XSCS_TILE")) {
        int t0, t1, t2;
        if (sscanf(e, "%d,%d,%d", &t0, &t1, &t2) == 3 && t0 > 0 && t1 > 0 && t2 > 0 && t0 * t1 * t2 <= 1024 &&
            (int64_t)(t0 + 2 * rx) * (t1 + 2 * ry) * (t2 + 2 * rz) * 8 <= 64 * 1024) {
            best[0] = t0; best[1] = t1; best[2] = t2;
        }
    }
    if (!best[0]) return false;
    m.xscs_steps.assign(3 * Kp, 0);  // padding offsets: the row itself
    for (int k = 0; k < K; k++) {
        m.xscs_steps[3 * k] = dx[k];
        m.xscs_steps[3 * k + 1] = dy[k];
        m.xscs_steps[3 * k + 2] = dz[k];
    }
    m.xscs_r[0] = rx; m.xscs_r[1] = ry; m.xscs_r[2] = rz;
    m.xscs = true;
    xscs_set_tile(m, best);
    return true;
}

// Class of every row of [r0, r1): rows with the same (col - base[i], value bits) list share
// one; hashed in parallel, grouped serially with a full comparison.  Returns the
// number of classes (ids in cls, one representative row per class in rep), or
// -1 past 65536.
static int64_t row_classes(const std::vector<int64_t> &rp, const std::vector<int32_t> &col,
                           const std::vector<double> &val, const std::vector<int64_t> &base, int64_t r0,
                           int64_t r1, std::vector<uint16_t> &cls, std::vector<int64_t> &rep) {
    const int64_t n = (int64_t)rp.size() - 1;
    std::vector<uint64_t> h(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = r0; i < r1; i++) {
        uint64_t x = 0x9E3779B97F4A7C15ull ^ (uint64_t)(rp[i + 1] - rp[i]);
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            uint64_t bits;
            std::memcpy(&bits, &val[e], 8);
            x = (x ^ (uint64_t)(uint32_t)((int64_t)col[e] - base[i])) * 0x100000001B3ull;
            x = (x ^ bits) * 0xFF51AFD7ED558CCDull;
            x ^= x >> 29;
        }
        h[i] = x;
    }
    auto same_row = [&](int64_t i, int64_t j) {
        if (rp[i + 1] - rp[i] != rp[j + 1] - rp[j]) return false;
        for (int64_t a = rp[i], b = rp[j]; a < rp[i + 1]; a++, b++) {
            if ((int64_t)col[a] - base[i] != (int64_t)col[b] - base[j]) return false;
            if (std::memcmp(&val[a], &val[b], 8) != 0) return false;
        }
        return true;
    };
    std::unordered_map<uint64_t, std::vector<int32_t>> by_hash;  // hash -> classes (collisions chained)
    rep.clear();
    cls.assign(n, 0);
    for (int64_t i = r0; i < r1; i++) {
        auto &cands = by_hash[h[i]];
        int32_t c = -1;
        for (int32_t q : cands)
            if (same_row(rep[q], i)) { c = q; break; }
        if (c < 0) {
            c = (int32_t)rep.size();
            if (c >= 65536) return -1;
            rep.push_back(i);
            cands.push_back(c);
        }
        cls[i] = (uint16_t)c;
    }
    return (int64_t)rep.size();
}

static void spmv_xscs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
                      hipStream_t s, int64_t seg = -1);

// Pick the tile by timing the candidates on the device (a few SET launches each
// on scratch vectors): the modelled choice missed by up to 1.6x -- wide x rows
// stage with fewer, longer loads, but a tile whose waves straddle boundary
// classes reads the dictionary per lane (profiles/r03/ab_xscs_*.log).  The
// tile changes no result (same sums in the same order).
static void xscs_autotune(GpuCsr &m) {
    if (getenv("FAMG_XSCS_TILE")) {
        m.xscs_tile_src = TUNE_ENV;
        return;
    }
    const int64_t nx = m.grid[0], ny = m.grid[1], nz = m.grid[2], n = m.nrows;
    const int rx = m.xscs_r[0], ry = m.xscs_r[1], rz = m.xscs_r[2];
    // a shape of the frozen table (tuning.cpp) takes its tile without timing
    const TileKey key{nx, ny, nz, rx, ry, rz, (int)m.scs_kr, m.scs_nclass, m.rframe.on()};
    {
        int t[3];
        if (getenv("FAMG_TUNE_RETIME") == nullptr && tune_tile_lookup(key, t)) {
            xscs_set_tile(m, t);
            m.xscs_tile_src = TUNE_TABLE;
            tune_tile_record(key, t, TUNE_TABLE);
            return;
        }
    }
    std::vector<std::array<int, 3>> cands;
    for (int tx : {4, 8, 16, 32, 64})
        for (int ty : {1, 2, 4, 8, 16})
            for (int tz : {1, 2, 4, 8}) {
                if (tx > nx || ty > ny || tz > nz) continue;
                const int64_t T = (int64_t)tx * ty * tz;
                const int64_t W = (int64_t)(tx + 2 * rx) * (ty + 2 * ry) * (tz + 2 * rz);
                if (T < std::min<int64_t>(64, n) || T > 1024 || W * 8 > 64 * 1024) continue;
                if (T < 128 && n >= 1024 * 256) continue;
                if (tx < 8 && nx >= 8) continue;  // short x rows stage poorly (ab_xscs)
                cands.push_back({tx, ty, tz});
            }
    if (cands.size() < 2) return;
    hipStream_t s = m.ctx->stream;
    DevBuf<double> x(m.ncols), y(m.nrows);
    FAMG_CHECK_HIP(hipMemsetAsync(x.get(), 0, m.ncols * sizeof(double), s));
    hipEvent_t e0, e1;
    FAMG_CHECK_HIP(hipEventCreate(&e0));
    FAMG_CHECK_HIP(hipEventCreate(&e1));
    int best[3] = {m.xscs_t[0], m.xscs_t[1], m.xscs_t[2]};
    float best_ms = 1e30f;
    for (const auto &c : cands) {
        xscs_set_tile(m, c.data());
        spmv_xscs(m, x.get(), y.get(), SPMV_SET, SpmvEpi{}, s);
        FAMG_CHECK_HIP(hipEventRecord(e0, s));
        for (int r = 0; r < 3; r++) spmv_xscs(m, x.get(), y.get(), SPMV_SET, SpmvEpi{}, s);
        FAMG_CHECK_HIP(hipEventRecord(e1, s));
        FAMG_CHECK_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        FAMG_CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_ms) {
            best_ms = ms;
            best[0] = c[0]; best[1] = c[1]; best[2] = c[2];
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    xscs_set_tile(m, best);
    m.xscs_tile_src = TUNE_TIMED;
    tune_tile_record(key, best, TUNE_TIMED);
}

bool build_scs(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes) {
    scs_release(m);
    if (g_spmv_format_policy != 0 || scs_disabled() || m.no_sellp || m.nrows < 1024 || m.nnz == 0 ||
        m.ncols < m.nrows)
        return false;
    const int64_t n = m.nrows;
    // a rank-local matrix of a distributed grid level with its slab frames: its
    // columns map to grid planes (ghost planes included), so the whole matrix
    // can run x-staged through the frame -- and only that way
    const SlabFrame &F = m.cframe;
    const bool framed = F.on() && m.rframe.on();
    if (framed && (m.rframe.nx != F.nx || m.rframe.ny != F.ny || m.rframe.z0 != F.z0 || m.rframe.nz != F.nz ||
                   n != F.n_own() || m.ncols != F.n_own() + (F.gl + F.gh) * F.pl() ||
                   m.grid[0] != F.nx || m.grid[1] != F.ny || m.grid[2] != F.nz))
        return false;
    // the whole matrix (square), or the longest row segment of a [owned | ghost]
    // distributed level when its rows read owned columns only (the halo interior)
    int64_t r0 = 0, r1 = n, seg = -1;
    if (m.nrows != m.ncols && !framed) {
        if (m.seg_rows.size() < 3) return false;
        seg = 0;
        for (size_t g = 1; g + 1 < m.seg_rows.size(); g++)
            if (m.seg_rows[g + 1] - m.seg_rows[g] > m.seg_rows[seg + 1] - m.seg_rows[seg]) seg = (int64_t)g;
        r0 = m.seg_rows[seg];
        r1 = m.seg_rows[seg + 1];
        if (r1 - r0 < 1024 || (m.has_dia() && m.dia_seg == seg)) return false;
        other_bytes = (int64_t)((double)other_bytes * (double)(r1 - r0) / (double)n);
    }
    hipStream_t st = m.ctx->stream;
    std::vector<int32_t> col(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    if (seg >= 0)
        for (int64_t e = rp[r0]; e < rp[r1]; e++)
            if (col[e] >= n) return false;  // a ghost column
    if (framed) {  // local column -> position in the contiguous plane frame (ghosts below negative)
        const int64_t own = F.n_own(), below = F.gl * F.pl();
#pragma omp parallel for schedule(static)
        for (int64_t e = 0; e < m.nnz; e++) {
            const int64_t c = col[e];
            col[e] = (int32_t)(c < own ? c : c - own < below ? c - own - below : c - below);
        }
    }
    // union of the offsets: bounded first (K <= SCS_KMAX), then a bitmap over the span
    int64_t omin = INT64_MAX, omax = INT64_MIN;
#pragma omp parallel for reduction(min : omin) reduction(max : omax) schedule(static)
    for (int64_t i = r0; i < r1; i++)
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int64_t o = (int64_t)col[e] - i;
            omin = std::min(omin, o);
            omax = std::max(omax, o);
        }
    const int64_t span = omax - omin + 1;
    if (span > (int64_t(1) << 26)) return false;
    std::vector<uint8_t> seen(span, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = r0; i < r1; i++)
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) seen[(int64_t)col[e] - i - omin] = 1;  // benign same-value race
    std::vector<int32_t> offs;
    for (int64_t o = 0; o < span; o++)
        if (seen[o]) {
            offs.push_back((int32_t)(o + omin));
            if ((int64_t)offs.size() > SCS_KMAX) return false;
        }
    const int K = (int)offs.size();
    if (K == 0 || (double)K * (double)(r1 - r0) > 2.0 * (double)(rp[r1] - rp[r0])) return false;  // mostly padding
    // on a grid the x-staged kernel may take the operator (checked below);
    // otherwise short stencils stay on SELL-64: A_1 of the 256^3 cycle (33
    // offsets, 8-bit codes) ran 47 vs 44 us here; A_2 (179 offsets, 16-bit
    // codes) 31-46 vs 55 us
    const bool on_grid = framed ? xscs_enabled() : seg < 0 && grid_applies(m);
    if (K < (on_grid ? 8 : SCS_KMIN)) return false;
    // operators with a <= 256-entry value table keep SELL-64, whose codes decode
    // from an LDS table: A_1 of the 27-pt cycle (125 offsets, 8-bit codes) ran
    // 135 vs 121 us here (two dictionary loads per step per row pair)
    bool small_table = false;
    {
        std::vector<unsigned long long> tab;
        const int vb = csr_value_table(m, tab);
        small_table = vb == 4 || vb == 8;
        if (small_table && !on_grid) return false;
    }
    std::vector<double> val(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), m.val.get(), m.nnz * sizeof(double), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> base(n);
    for (int64_t i = 0; i < n; i++) base[i] = i;
    std::vector<uint16_t> cls;
    std::vector<int64_t> rep;
    if (row_classes(rp, col, val, base, r0, r1, cls, rep) < 0) return false;
    const int64_t C = (int64_t)rep.size();
    const int Kp = (K + SCS_U - 1) / SCS_U * SCS_U;
    const int ib = C <= 256 ? 1 : 2;
    const int64_t dict_bytes = (int64_t)Kp * C * 8;
    const int64_t stream = ib * (r1 - r0) + dict_bytes + 4 * Kp;
    // x staged per grid tile when the offsets are grid steps within the grid
    // FAMG_SCS_ROWS=1: few long rows take the lanes-per-row kernel even where the
    // x-staged one applies (A/B)
    const bool rows_pref = scs_rows_pref() && r1 - r0 < SCS_LANES_ROWS && Kp >= 256 && !framed;
    const bool xs3 = !rows_pref && on_grid && dict_bytes <= (int64_t(256) << 20) &&
                     (framed || (double)stream <= 0.5 * (double)other_bytes) && xscs_setup(m, offs, Kp, rp, col, val);
    if (!xs3 && (K < SCS_KMIN || small_table || framed)) return false;
    // few long rows: one row per wave, the dictionary streamed (up to 256 MiB)
    const bool lanes = !xs3 && r1 - r0 < SCS_LANES_ROWS && Kp >= 256;
    if (lanes && !scs_lanes_enabled()) { scs_release(m); return false; }
    if (!xs3 && (dict_bytes > (int64_t(lanes ? 256 : 16) << 20) || (double)stream > 0.5 * (double)other_bytes))
        return false;
    std::vector<double> dict((size_t)Kp * C, 0.0);
    for (int64_t c = 0; c < C; c++) {
        const int64_t i = rep[c];
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int32_t o = (int32_t)((int64_t)col[e] - i);
            const int k = (int)(std::lower_bound(offs.begin(), offs.end(), o) - offs.begin());
            dict[(size_t)c * Kp + k] = val[e];
        }
    }
    offs.resize(Kp, 0);  // padding offsets: value +0.0 at the row itself
    m.scs_offs.resize(Kp);
    m.scs_dict.resize((size_t)Kp * C);
    m.scs_cls.resize(n * ib);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.scs_offs.get(), offs.data(), Kp * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.scs_dict.get(), dict.data(), dict.size() * 8, hipMemcpyHostToDevice, st));
    if (ib == 1) {
        std::vector<uint8_t> c8(n);
        for (int64_t i = 0; i < n; i++) c8[i] = (uint8_t)cls[i];
        FAMG_CHECK_HIP(hipMemcpyAsync(m.scs_cls.get(), c8.data(), n, hipMemcpyHostToDevice, st));
        FAMG_CHECK_HIP(hipStreamSynchronize(st));
    } else {
        FAMG_CHECK_HIP(hipMemcpyAsync(m.scs_cls.get(), cls.data(), n * 2, hipMemcpyHostToDevice, st));
        FAMG_CHECK_HIP(hipStreamSynchronize(st));
    }
    m.scs_k = Kp;
    m.scs_kr = K;
    m.scs_nclass = C;
    m.scs_ib = ib;
    m.scs_seg = seg;
    m.scs_lanes = lanes;
    if (m.xscs) xscs_autotune(m);
    return true;
}

static void spmv_xscs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
                      hipStream_t s, int64_t seg) {
    XscsArgs a{};
    a.cls = m.scs_cls.get();
    a.dict = m.scs_dict.get();
    a.lo = m.xscs_lo.get();
    a.k = (int32_t)m.scs_k;
    a.kr = (int32_t)m.scs_kr;
    a.nx = (int)m.grid[0]; a.ny = (int)m.grid[1]; a.nz = (int)m.grid[2];
    a.tx = m.xscs_t[0]; a.ty = m.xscs_t[1]; a.tz = m.xscs_t[2];
    a.rx = m.xscs_r[0]; a.ry = m.xscs_r[1]; a.rz = m.xscs_r[2];
    a.wx = a.tx + 2 * a.rx; a.wy = a.ty + 2 * a.ry; a.wz = a.tz + 2 * a.rz;
    a.ws = m.xscs_ws;
    FAMG_REQUIRE(a.ws >= a.wx, AMG_ERR_UNSUPPORTED, "x-staged classes: no window stride");
    a.ntx = (int)ceil_div(a.nx, a.tx); a.nty = (int)ceil_div(a.ny, a.ty);
    const int ntz = (int)ceil_div(a.nz, a.tz);
    a.rwx = 1.0f / (float)a.wx; a.rwy = 1.0f / (float)a.wy;
    a.rtx = 1.0f / (float)a.tx; a.rty = 1.0f / (float)a.ty;
    FAMG_REQUIRE(m.xscs_fdiv, AMG_ERR_UNSUPPORTED, "x-staged classes: window too large for the float divisions");
    a.zlo = 0; a.zhi = a.nz; a.add_lo = a.add_hi = 0;
    const SlabFrame &F = m.cframe;
    if (F.on()) {  // rank-local: the ghost planes below / above the owned ones
        a.zlo = (int)-F.gl;
        a.zhi = (int)(F.nz + F.gh);
        a.add_lo = F.add_lo();
        a.add_hi = F.add_hi();
        FAMG_REQUIRE(mode != SPMV_RESID0 || F.gl + F.gh == 0, AMG_ERR_UNSUPPORTED,
                     "x-staged classes: the folded residual needs d on the ghost planes");
    }
    // z-tiles of this launch: all, or (segments of a rank-local matrix) 1 = the
    // tiles whose window lies in the owned planes, 0 / 2 = those before / after
    int tz0 = 0, tz1 = ntz;
    if (seg >= 0 && F.on()) {  // a window reads ghosts only where it crosses into a ghost plane
        auto below = [&](int t) { return t * a.tz - a.rz < 0 && F.gl > 0; };
        auto above = [&](int t) { return (t + 1) * a.tz + a.rz > a.nz && F.gh > 0; };
        int ta = 0;
        while (ta < ntz && below(ta)) ta++;
        int tb = ta;
        while (tb < ntz && !above(tb)) tb++;
        tz0 = seg == 0 ? 0 : seg == 1 ? ta : tb;
        tz1 = seg == 0 ? ta : seg == 1 ? tb : ntz;
    }
    if (tz1 <= tz0) return;
    a.tile0 = a.ntx * a.nty * tz0;
    a.x = x; a.y = y; a.b = epi.b; a.d = epi.d; a.dc = epi.dc; a.dt = epi.dt;
    const int T = a.tx * a.ty * a.tz;
    const int rl = T <= 256 ? 1 : T <= 512 ? 2 : 4;
    const size_t lds = (size_t)a.ws * a.wy * a.wz * sizeof(double);
    const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * (tz1 - tz0))), block(256);
#define FAMG_XS3(M, IB)                                                                            \
    if (rl == 1) spmv_xscs_kernel<M, IB, 1><<<grid, block, lds, s>>>(a);                           \
    else if (rl == 2) spmv_xscs_kernel<M, IB, 2><<<grid, block, lds, s>>>(a);                      \
    else spmv_xscs_kernel<M, IB, 4><<<grid, block, lds, s>>>(a);
#define FAMG_XS3M(IB)                                                                              \
    switch (mode) {                                                                                \
    case SPMV_SET: FAMG_XS3(SPMV_SET, IB) break;                                                   \
    case SPMV_ADD: FAMG_XS3(SPMV_ADD, IB) break;                                                   \
    case SPMV_RESID: FAMG_XS3(SPMV_RESID, IB) break;                                               \
    case SPMV_RESID0: FAMG_XS3(SPMV_RESID0, IB) break;                                             \
    case SPMV_JACOBI: FAMG_XS3(SPMV_JACOBI, IB) break;                                             \
    default: fail(AMG_ERR_UNSUPPORTED, "stencil-class storage: unsupported SpMV epilogue");        \
    }
    if (m.scs_ib == 1) { FAMG_XS3M(1) }
    else { FAMG_XS3M(2) }
#undef FAMG_XS3M
#undef FAMG_XS3
    FAMG_CHECK_HIP(hipGetLastError());
}

void spmv_scs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg) {
    if (m.xscs && (seg < 0 || m.cframe.on())) {  // a framed matrix: segments are z-tile ranges, not row ranges
        spmv_xscs(m, x, y, mode, epi, s, seg);
        return;
    }
    const int64_t r0 = seg < 0 ? 0 : m.seg_rows[seg];
    const int64_t r1 = seg < 0 ? m.nrows : m.seg_rows[seg + 1];
    if (r1 <= r0) return;
    ScsArgs a{m.scs_cls.get(), m.scs_dict.get(), m.scs_offs.get(), (int32_t)m.scs_k, (int32_t)m.scs_nclass,
              (int32_t)r0, (int32_t)r1, (int32_t)m.ncols, x, y, epi.b, epi.d, epi.dc, epi.dt};
    const dim3 grid((unsigned)ceil_div(r1 - r0, m.scs_lanes ? 4 : 512)), block(256);
#define FAMG_SCS2(M, IB)                                                                           \
    if (m.scs_lanes) spmv_scs_lanes_kernel<M, IB><<<grid, block, 0, s>>>(a);                       \
    else spmv_scs_kernel<M, IB><<<grid, block, 0, s>>>(a);
#define FAMG_SCS(IB)                                                                               \
    switch (mode) {                                                                                \
    case SPMV_SET: FAMG_SCS2(SPMV_SET, IB) break;                                                  \
    case SPMV_ADD: FAMG_SCS2(SPMV_ADD, IB) break;                                                  \
    case SPMV_RESID: FAMG_SCS2(SPMV_RESID, IB) break;                                              \
    case SPMV_JACOBI: FAMG_SCS2(SPMV_JACOBI, IB) break;                                            \
    default: fail(AMG_ERR_UNSUPPORTED, "stencil-class storage: unsupported SpMV epilogue");        \
    }
    if (m.scs_ib == 1) { FAMG_SCS(1) }
    else { FAMG_SCS(2) }
#undef FAMG_SCS
#undef FAMG_SCS2
    FAMG_CHECK_HIP(hipGetLastError());
}


}  // namespace famg
