// spmm.hip -- multi-RHS SpMM Y = A X for the compressed storages (SURVEY.md
// 8(f) f2: the k-wide applies of near-null smoothing and the error propagator,
// adaptivity.rs:168-244,307-390, hierarchy.rs:219-226).
//
// The SELL-64 SpMM (spmv.hip) covers fp64-valued SELL; here the storages the
// hierarchies actually use: DIA codes (constant-stencil operators, incl. the
// 33- and 27-diagonal run patterns), stencil classes (structured Galerkin
// levels) and 3x3 blocks (elasticity / C5).  Each kernel reads a row's matrix
// data once per group of up to 8 columns and, per column, sums exactly the
// terms the single-vector kernel of that storage sums, in the same order
// (ascending diagonals / offsets / block columns, fma from 0.0; the lanes-per-
// row class kernel with the same lane split and butterfly), so every column is
// bitwise the single-vector SpMV.  Column-major X, Y with leading dimensions.
#include <algorithm>
#include <type_traits>

#include "famg.hpp"

namespace famg {

constexpr int SPMM_COLS = 8;  // columns per launch

typedef double spmm_dbl2_t __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ DIA codes

struct SpmmDiaArgs {
    const uint32_t *codes;
    const double *vtab;
    int32_t ntab, k, nrows, ncols;
    int32_t off[64];
    const double *x;
    int64_t ldx;
    double *y;
    int64_t ldy;
};

// one row per lane: the row's code words once, then per column the K terms
// fma(value, x[clamp(row + off_k)], acc) (padding terms carry +0.0 codes)
template <int VB, int CW, int KB>
__global__ __launch_bounds__(256) void spmm_dia_kernel(SpmmDiaArgs a) {
    __shared__ double stab[VB == 4 ? 16 : 256];
    for (int q = threadIdx.x; q < a.ntab; q += 256) stab[q] = a.vtab[q];
    __syncthreads();
    constexpr uint32_t MASK = (1u << VB) - 1;
    const int row = (int)(xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x);
    if (row >= a.nrows) return;
    uint32_t w[CW];
#pragma unroll
    for (int q = 0; q < CW; q++) w[q] = __builtin_nontemporal_load(a.codes + (int64_t)row * CW + q);
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c] = 0.0;
    for (int k = 0; k < a.k; k++) {
        const double v = stab[(w[(k * VB) >> 5] >> ((k * VB) & 31)) & MASK];
        const int64_t col = min(max(row + a.off[k], 0), a.ncols - 1);
#pragma unroll
        for (int c = 0; c < KB; c++) acc[c] = fma(v, a.x[col + c * a.ldx], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < KB; c++) a.y[row + c * a.ldy] = acc[c];
}

// ----------------------------------------------------------- stencil classes

struct SpmmScsArgs {
    const void *cls;
    const double *dict;
    const int32_t *offs;
    int32_t k, nrows, ncols;
    const double *x;
    int64_t ldx;
    double *y;
    int64_t ldy;
};

template <int IB> __device__ __forceinline__ int spmm_cls(const void *cls, int r) {
    return IB == 1 ? (int)static_cast<const uint8_t *>(cls)[r] : (int)static_cast<const uint16_t *>(cls)[r];
}

// one row per lane (spmv_scs_kernel's order: the K offsets ascending, clamped x)
template <int IB, int KB>
__global__ __launch_bounds__(256) void spmm_scs_kernel(SpmmScsArgs a) {
    const int row = (int)(xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x);
    if (row >= a.nrows) return;
    const double *dct = a.dict + (int64_t)spmm_cls<IB>(a.cls, row) * a.k;
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c] = 0.0;
    for (int k = 0; k < a.k; k++) {
        const double v = dct[k];
        const int64_t col = min(max(row + a.offs[k], 0), a.ncols - 1);
#pragma unroll
        for (int c = 0; c < KB; c++) acc[c] = fma(v, a.x[col + c * a.ldx], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < KB; c++) a.y[row + c * a.ldy] = acc[c];
}

// one row per wave (spmv_scs_lanes_kernel's order: lane q takes offsets q,
// q + 64, ... in groups of 8 steps, +0.0 past K, then the xor butterfly)
template <int IB, int KB>
__global__ __launch_bounds__(256) void spmm_scs_lanes_kernel(SpmmScsArgs a) {
    const int row = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (int)(threadIdx.x >> 6));
    if (row >= a.nrows) return;
    const int lane = threadIdx.x & 63;
    const double *dct = a.dict + (int64_t)spmm_cls<IB>(a.cls, row) * a.k;
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c] = 0.0;
    int k0 = 0;
    for (; k0 + 8 * 64 <= a.k; k0 += 8 * 64) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int k = k0 + 64 * u + lane;
            const double v = dct[k];
            const int64_t col = min(max(row + a.offs[k], 0), a.ncols - 1);
#pragma unroll
            for (int c = 0; c < KB; c++) acc[c] = fma(v, a.x[col + c * a.ldx], acc[c]);
        }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int k = k0 + 64 * u + lane;
        const int kc = min(k, a.k - 1);
        const double v = k < a.k ? dct[kc] : 0.0;
        const int64_t col = min(max(row + a.offs[kc], 0), a.ncols - 1);
#pragma unroll
        for (int c = 0; c < KB; c++) acc[c] = fma(v, a.x[col + c * a.ldx], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < KB; c++) {
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) acc[c] += __shfl_xor(acc[c], m);
    }
    if (lane == 0) {
#pragma unroll
        for (int c = 0; c < KB; c++) a.y[row + c * a.ldy] = acc[c];
    }
}

// --------------------------------------------------------------- 3x3 blocks

constexpr int64_t SPMM_BSR_STEP = 64 * (9 * 8 + 4);  // bsr.hip's 4864-B block step
constexpr int SPMM_BSR_K8 = 4 * 64 * 16;
constexpr int SPMM_BSR_COL = SPMM_BSR_K8 + 64 * 8;

struct SpmmBsrArgs {
    const char *data;
    const int32_t *row0, *soff;
    int32_t nslices;
    const double *x;
    int64_t ldx;
    double *y;
    int64_t ldy;
};

// one node row per lane (spmv_bsr3_kernel's order: blocks ascending, dof row
// r of block J sums v(r,0) x(3J), v(r,1) x(3J+1), v(r,2) x(3J+2) with fma)
template <int KB>
__global__ __launch_bounds__(256) void spmm_bsr3_kernel(SpmmBsrArgs a) {
    const int sl = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int lane = threadIdx.x & 63;
    const int I = a.row0[sl] + lane;
    const bool live = I < a.row0[sl + 1];
    const int t0 = a.soff[sl], w = a.soff[sl + 1] - t0;
    double acc[KB][3];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c][0] = acc[c][1] = acc[c][2] = 0.0;
    for (int t = 0; t < w; t++) {
        const char *p = a.data + (int64_t)(t0 + t) * SPMM_BSR_STEP;
        double v[9];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const spmm_dbl2_t u = __builtin_nontemporal_load(reinterpret_cast<const spmm_dbl2_t *>(p + q * 1024) + lane);
            v[2 * q] = u.x;
            v[2 * q + 1] = u.y;
        }
        v[8] = __builtin_nontemporal_load(reinterpret_cast<const double *>(p + SPMM_BSR_K8) + lane);
        const int J = __builtin_nontemporal_load(reinterpret_cast<const int32_t *>(p + SPMM_BSR_COL) + lane);
#pragma unroll
        for (int c = 0; c < KB; c++) {
            const double *xp = a.x + 3 * (int64_t)J + c * a.ldx;
            const double x0 = xp[0], x1 = xp[1], x2 = xp[2];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                acc[c][r] = fma(v[3 * r], x0, acc[c][r]);
                acc[c][r] = fma(v[3 * r + 1], x1, acc[c][r]);
                acc[c][r] = fma(v[3 * r + 2], x2, acc[c][r]);
            }
        }
    }
    if (live) {
#pragma unroll
        for (int c = 0; c < KB; c++)
#pragma unroll
            for (int r = 0; r < 3; r++) a.y[3 * (int64_t)I + r + c * a.ldy] = acc[c][r];
    }
}

// ------------------------------------------------------------- pattern SELL

struct SpmmSellpArgs {
    const char *vals;
    const int64_t *eoff;
    const int32_t *row0;
    const int2 *pat;
    const int32_t *offs;
    const int32_t *rbase;
    const double *vtab;
    int32_t ntab, nslices, ncols;
    const double *x;
    int64_t ldx;
    double *y;
    int64_t ldy;
};

// spmv_sellp_kernel's sums per column: lane q of a row walks its steps t = s L + q
// ascending with fma (fp64 values or 4/8-bit codes from the LDS table), padding
// steps +0.0 at a clamped column, then the same xor butterfly over the L lanes.
// A wave per slice.
template <int L, int VB, int KB>
__global__ __launch_bounds__(256) void spmm_sellp_kernel(SpmmSellpArgs a) {
    __shared__ double stab[VB ? 256 : 1];
    if constexpr (VB != 0) {
        for (int i = threadIdx.x; i < a.ntab; i += 256) stab[i] = a.vtab[i];
        __syncthreads();
    }
    const int s = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (int)(threadIdx.x >> 6));
    if (s >= a.nslices) return;
    const int lane = threadIdx.x & 63, r = lane / L, q = lane % L;
    const int row = a.row0[s] + r;
    const bool live = row < a.row0[s + 1];
    const int rowc = live ? row : a.row0[s];
    const int base = a.rbase ? a.rbase[rowc] : rowc;
    const int2 pw = a.pat[s];
    const int32_t *off = a.offs + pw.x;
    const int w = pw.y, S = (w + L - 1) / L;
    const int64_t e0 = a.eoff[s];
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; c++) acc[c] = 0.0;
    // codes: whole words of K lane-steps, as spmv_sellp_kernel walks them
    const int send = VB == 0 ? S : (S + 32 / (VB ? VB : 1) - 1) / (32 / (VB ? VB : 1)) * (32 / (VB ? VB : 1));
    for (int st = 0; st < send; st++) {
        const int t = st * L + q;
        const bool in = t < w;
        const int64_t col = min(max(base + off[in ? t : 0], 0), a.ncols - 1);
        double v;
        if constexpr (VB == 0) {
            v = __builtin_nontemporal_load(reinterpret_cast<const double *>(a.vals) + e0 + (int64_t)st * 64 + lane);
        } else {
            constexpr int K = 32 / VB;
            const uint32_t wd = reinterpret_cast<const uint32_t *>(a.vals)[e0 + (int64_t)(st / K) * 64 + lane];
            v = stab[(wd >> ((st % K) * VB)) & ((1u << VB) - 1)];
        }
        v = in ? v : 0.0;
#pragma unroll
        for (int c = 0; c < KB; c++) acc[c] = fma(v, (L > 1 || VB == 0 || in) ? a.x[col + c * a.ldx] : 0.0, acc[c]);
    }
#pragma unroll
    for (int c = 0; c < KB; c++)
#pragma unroll
        for (int m = L / 2; m > 0; m >>= 1) acc[c] += __shfl_xor(acc[c], m);
    if (live && q == 0) {
#pragma unroll
        for (int c = 0; c < KB; c++) a.y[row + c * a.ldy] = acc[c];
    }
}

// ------------------------------------------------------------------ dispatch

#define FAMG_SPMM_KB(KB_EXPR, LAUNCH)                                                              \
    switch (KB_EXPR) {                                                                             \
    case 1: LAUNCH(1); break;                                                                      \
    case 2: LAUNCH(2); break;                                                                      \
    case 3: LAUNCH(3); break;                                                                      \
    case 4: LAUNCH(4); break;                                                                      \
    case 5: LAUNCH(5); break;                                                                      \
    case 6: LAUNCH(6); break;                                                                      \
    case 7: LAUNCH(7); break;                                                                      \
    default: LAUNCH(8); break;                                                                     \
    }

// Y = A X over k columns for DIA / stencil-class / 3x3-block storage; false if
// the storage is none of these (the caller applies per column).
bool spmm_compressed(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k, hipStream_t s) {
    const bool dia = m.kernel == SPMV_KERNEL_DIA && m.has_dia() && !m.dia_rowid && m.dia_r0 == 0 &&
                     m.dia_r1 == m.nrows && m.dia_k <= 64;
    const bool scs = m.kernel == SPMV_KERNEL_SCS && m.has_scs() && m.scs_seg < 0;
    const bool bsr = m.kernel == SPMV_KERNEL_BSR && m.has_bsr();
    const bool xs = m.kernel == SPMV_KERNEL_XS && m.has_xs();
    const int sL = m.sellp_L, sV = m.sellp_vbits;
    const bool sellp = m.kernel == SPMV_KERNEL_SELLP && m.has_sellp() && m.sellp_seg_slc.size() <= 2 &&
                       (sL == 1 || sL == 2 || sL == 4 || sL == 8 || sL == 16 || sL == 32 || sL == 64) &&
                       (sV == 0 || sV == 4 || sV == 8);
    if (xs) return spmm_xs(m, x, ldx, y, ldy, k, s);  // xsell.hip: per column with its x chunks in LDS
    if (!dia && !scs && !bsr && !sellp) return false;
    if (m.nrows == 0 || k == 0) return true;
    for (int64_t c0 = 0; c0 < k; c0 += SPMM_COLS) {
        const int kb = (int)std::min<int64_t>(SPMM_COLS, k - c0);
        const double *xc = x + c0 * ldx;
        double *yc = y + c0 * ldy;
        if (dia) {
            SpmmDiaArgs a{};
            a.codes = m.dia_codes.get();
            a.vtab = m.dia_vtab.get();
            a.ntab = (int32_t)m.dia_ntab;
            a.k = m.dia_k;
            a.nrows = (int32_t)m.nrows;
            a.ncols = (int32_t)m.ncols;
            for (int q = 0; q < m.dia_k; q++) a.off[q] = m.dia_off[q];
            a.x = xc;
            a.ldx = ldx;
            a.y = yc;
            a.ldy = ldy;
            const dim3 grid((unsigned)ceil_div(m.nrows, 256)), block(256);
            const int key = m.dia_vbits * 16 + m.dia_cw;
#define FAMG_L41(KB) spmm_dia_kernel<4, 1, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L42(KB) spmm_dia_kernel<4, 2, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L44(KB) spmm_dia_kernel<4, 4, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L45(KB) spmm_dia_kernel<4, 5, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L81(KB) spmm_dia_kernel<8, 1, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L82(KB) spmm_dia_kernel<8, 2, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L84(KB) spmm_dia_kernel<8, 4, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L88(KB) spmm_dia_kernel<8, 8, KB><<<grid, block, 0, s>>>(a)
#define FAMG_L89(KB) spmm_dia_kernel<8, 9, KB><<<grid, block, 0, s>>>(a)
            switch (key) {
            case 4 * 16 + 1: FAMG_SPMM_KB(kb, FAMG_L41) break;
            case 4 * 16 + 2: FAMG_SPMM_KB(kb, FAMG_L42) break;
            case 4 * 16 + 4: FAMG_SPMM_KB(kb, FAMG_L44) break;
            case 4 * 16 + 5: FAMG_SPMM_KB(kb, FAMG_L45) break;
            case 8 * 16 + 1: FAMG_SPMM_KB(kb, FAMG_L81) break;
            case 8 * 16 + 2: FAMG_SPMM_KB(kb, FAMG_L82) break;
            case 8 * 16 + 4: FAMG_SPMM_KB(kb, FAMG_L84) break;
            case 8 * 16 + 8: FAMG_SPMM_KB(kb, FAMG_L88) break;
            case 8 * 16 + 9: FAMG_SPMM_KB(kb, FAMG_L89) break;
            default: fail(AMG_ERR_INVALID, "SpMM: unsupported DIA code layout");
            }
        } else if (scs) {
            SpmmScsArgs a{m.scs_cls.get(), m.scs_dict.get(), m.scs_offs.get(), (int32_t)m.scs_k,
                          (int32_t)m.nrows, (int32_t)m.ncols, xc, ldx, yc, ldy};
            const dim3 grid((unsigned)ceil_div(m.nrows, m.scs_lanes ? 4 : 256)), block(256);
#define FAMG_S1(KB) spmm_scs_kernel<1, KB><<<grid, block, 0, s>>>(a)
#define FAMG_S2(KB) spmm_scs_kernel<2, KB><<<grid, block, 0, s>>>(a)
#define FAMG_SL1(KB) spmm_scs_lanes_kernel<1, KB><<<grid, block, 0, s>>>(a)
#define FAMG_SL2(KB) spmm_scs_lanes_kernel<2, KB><<<grid, block, 0, s>>>(a)
            if (m.scs_lanes) {
                if (m.scs_ib == 1) { FAMG_SPMM_KB(kb, FAMG_SL1) }
                else { FAMG_SPMM_KB(kb, FAMG_SL2) }
            } else {
                if (m.scs_ib == 1) { FAMG_SPMM_KB(kb, FAMG_S1) }
                else { FAMG_SPMM_KB(kb, FAMG_S2) }
            }
        } else if (sellp) {
            SpmmSellpArgs a{m.sellp_vals.get(), m.sellp_eoff.get(), m.sellp_row0.get(),
                            reinterpret_cast<const int2 *>(m.sellp_pat.get()), m.sellp_offs.get(), m.sellp_rbase.get(),
                            m.sellp_vtab.get(), (int32_t)m.sellp_ntab, (int32_t)m.sellp_slices, (int32_t)m.ncols,
                            xc, ldx, yc, ldy};
            const dim3 grid((unsigned)ceil_div(m.sellp_slices, 4)), block(256);
#define FAMG_P(L, VB, KB) spmm_sellp_kernel<L, VB, KB><<<grid, block, 0, s>>>(a)
#define FAMG_PL(L, VB)                                                                              \
    {                                                                                               \
        auto go = [&](auto kbc) { FAMG_P(L, VB, decltype(kbc)::value); };                           \
        switch (kb) {                                                                               \
        case 1: go(std::integral_constant<int, 1>{}); break;                                        \
        case 2: go(std::integral_constant<int, 2>{}); break;                                        \
        case 3: go(std::integral_constant<int, 3>{}); break;                                        \
        case 4: go(std::integral_constant<int, 4>{}); break;                                        \
        case 5: go(std::integral_constant<int, 5>{}); break;                                        \
        case 6: go(std::integral_constant<int, 6>{}); break;                                        \
        case 7: go(std::integral_constant<int, 7>{}); break;                                        \
        default: go(std::integral_constant<int, 8>{}); break;                                       \
        }                                                                                           \
    }
#define FAMG_PV(L)                                                                                  \
    if (sV == 0) FAMG_PL(L, 0) else if (sV == 4) FAMG_PL(L, 4) else FAMG_PL(L, 8)
            switch (sL) {
            case 1: FAMG_PV(1) break;
            case 2: FAMG_PV(2) break;
            case 4: FAMG_PV(4) break;
            case 8: FAMG_PV(8) break;
            case 16: FAMG_PV(16) break;
            case 32: FAMG_PV(32) break;
            default: FAMG_PV(64) break;
            }
#undef FAMG_PV
#undef FAMG_PL
#undef FAMG_P
        } else {
            SpmmBsrArgs a{m.bsr_data.get(), m.bsr_row0.get(), m.bsr_soff.get(), (int32_t)m.bsr_slices,
                          xc, ldx, yc, ldy};
            const dim3 grid((unsigned)ceil_div(m.bsr_slices, 4)), block(256);
#define FAMG_B(KB) spmm_bsr3_kernel<KB><<<grid, block, 0, s>>>(a)
            FAMG_SPMM_KB(kb, FAMG_B)
        }
        FAMG_CHECK_HIP(hipGetLastError());
    }
    return true;
}

}  // namespace famg
