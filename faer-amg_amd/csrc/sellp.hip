// sellp.hip -- pattern SELL with L lanes per row for the dense Galerkin
// operators of structured hierarchies (A_2, A_3, A_4 of the 256^3 SA cycle:
// 168-1392 entries per row, 4K-262K rows).
//
// One lane per row (SELL-64) leaves these levels with 2-8 waves per SIMD and
// every wave walking 168+ dependent steps; the wave-per-row kernel has the waves
// but reads a 2-B column offset beside every value.  Here a slice is R = 64 / L
// consecutive rows, each row's steps dealt round-robin to its L lanes, and the
// columns are implicit: step t of row r is column r + off[t], off[] the sorted
// union of the slice's column offsets (col - row).  Slices share their offset
// list through a dictionary of patterns (interior rows of a constant-coefficient
// stencil all have the same one), so the matrix stream is the values alone
// (fp64; operators with a value table keep the value-code SELL-64, whose
// two-rows-per-lane 16-B code units measured faster).  Element (t, r) of a slice
// lies at (t / L) * 64 + r * L + t % L: every step group is one coalesced
// 64-element access.  Padding steps (a row without entry at an offset) hold
// +0.0 at a clamped in-range column.
//
// Summation order: lane q sums the steps t = q (mod L) ascending with fma, then
// the L partial sums are combined by a fixed butterfly -- deterministic, but not
// the oracle's sequential order (rounding-level differences, covered by the
// tolerance-based parity tests).  A_3 of the 256^3 cycle: 56 -> 46 us per SpMV
// against the wave-per-row kernel; A_2 with 16-bit codes: 91 vs 56 us for SELL-64.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>

#include "famg.hpp"

namespace famg {

struct SellpArgs {
    const char *vals;       // fp64 values or 8/16-bit codes
    const int64_t *eoff;    // per slice: first element
    const int32_t *row0;    // per slice: first row (+1 sentinel)
    const int32_t *pid;     // per slice: offset pattern
    const int32_t *poff;    // per pattern: start in offs (+1 sentinel)
    const int32_t *offs;    // concatenated sorted offset patterns
    const double *vtab;
    int32_t slice0, nslices, ncols;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
};

template <int VB> __device__ __forceinline__ double sellp_val(const SellpArgs &a, int64_t e) {
    if constexpr (VB == 0) return __builtin_nontemporal_load(reinterpret_cast<const double *>(a.vals) + e);
    else if constexpr (VB == 8) return a.vtab[__builtin_nontemporal_load(reinterpret_cast<const uint8_t *>(a.vals) + e)];
    else return a.vtab[__builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(a.vals) + e)];
}

// U step groups; every load of the group is issued before the fmas
template <int L, int VB, int U>
__device__ __forceinline__ void sellp_groups(const SellpArgs &a, int64_t e0, const int32_t *__restrict__ off, int w,
                                             int g0, int q, int row, int lane, double &acc) {
    double v[U], xx[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int t = (g0 + u) * L + q;
        const bool in = t < w;
        const int c = min(max(row + off[in ? t : 0], 0), a.ncols - 1);
        const double val = sellp_val<VB>(a, e0 + (int64_t)(g0 + u) * 64 + lane);
        v[u] = in ? val : 0.0;
        xx[u] = a.x[c];
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc = fma(v[u], xx[u], acc);
}

template <int MODE, int L, int VB>
__global__ __launch_bounds__(256) void spmv_sellp_kernel(SellpArgs a) {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int sl = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    if (sl >= a.nslices) return;
    const int s = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int r = lane / L, q = lane % L;
    const int row = a.row0[s] + r;
    const bool live = row < a.row0[s + 1];
    const int rowc = live ? row : a.row0[s];
    double br = 0.0, xr = 0.0, dr = 0.0, yr = 0.0;
    if (live && q == 0) {  // epilogue operands first
        if constexpr (MODE == SPMV_RESID) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
        if constexpr (MODE == SPMV_JACOBI) {
            xr = a.x[row];
            br = a.b[row];
            dr = a.dc ? a.dt[a.dc[row]] : a.d[row];
        }
    }
    const int p = a.pid[s];
    const int32_t *off = a.offs + a.poff[p];
    const int w = a.poff[p + 1] - a.poff[p];
    const int ng = (w + L - 1) / L;
    const int64_t e0 = a.eoff[s];
    double acc = 0.0;
    int g = 0;
    for (; g + 4 <= ng; g += 4) sellp_groups<L, VB, 4>(a, e0, off, w, g, q, rowc, lane, acc);
    switch (ng - g) {
    case 1: sellp_groups<L, VB, 1>(a, e0, off, w, g, q, rowc, lane, acc); break;
    case 2: sellp_groups<L, VB, 2>(a, e0, off, w, g, q, rowc, lane, acc); break;
    case 3: sellp_groups<L, VB, 3>(a, e0, off, w, g, q, rowc, lane, acc); break;
    default: break;
    }
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    if (live && q == 0) {
        if constexpr (MODE == SPMV_SET) a.y[row] = acc;
        else if constexpr (MODE == SPMV_ADD) a.y[row] = yr + acc;
        else if constexpr (MODE == SPMV_RESID) a.y[row] = br - acc;
        else a.y[row] = xr + dr * (br - acc);  // JACOBI
    }
}

static bool sellp_disabled() {
    static const bool off = [] {
        const char *e = getenv("FAMG_NO_SELLP");
        return e && e[0] == '1';
    }();
    return off;
}

// Builds the pattern-SELL storage of a square matrix whose rows average >= 48
// entries and whose slices share few offset patterns (a structured Galerkin
// operator); true if built.
bool build_sellp(GpuCsr &m, const std::vector<int64_t> &rp) {
    m.sellp_vals.release();
    m.sellp_eoff.release();
    m.sellp_row0.release();
    m.sellp_pid.release();
    m.sellp_poff.release();
    m.sellp_offs.release();
    m.sellp_vtab.release();
    m.sellp_slices = 0;
    m.sellp_elems = 0;
    m.sellp_L = 0;
    m.sellp_vbits = 0;
    m.sellp_seg_slc.clear();
    if (g_spmv_format_policy != 0 || sellp_disabled() || m.nrows != m.ncols || m.nrows < 1024 || m.nnz == 0)
        return false;
    const int64_t n = m.nrows;
    if (m.nnz < 48 * n) return false;
    // lanes per row: enough waves to fill the chip (>= 32K), >= 8 steps per lane
    const double avg = (double)m.nnz / (double)n;
    int L = 1;
    while (L < 64 && (n * L) / 64 < 32768 && avg / (2 * L) >= 8) L *= 2;
    if (L < 2) return false;
    const int R = 64 / L;
    hipStream_t st = m.ctx->stream;
    std::vector<int32_t> col(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    // slices of R rows inside the row segments; per slice the sorted union of offsets
    std::vector<int32_t> row0;
    std::vector<int64_t> seg_slc{0};
    for (size_t g = 0; g + 1 < m.seg_rows.size(); g++) {
        for (int64_t i = m.seg_rows[g]; i < m.seg_rows[g + 1]; i += R) row0.push_back((int32_t)i);
        seg_slc.push_back((int64_t)row0.size());
    }
    row0.push_back((int32_t)n);
    const int64_t ns = (int64_t)row0.size() - 1;
    std::vector<std::vector<int32_t>> pats;
    std::map<std::vector<int32_t>, int32_t> dict;
    std::vector<int32_t> pid(ns);
    int64_t elems = 0;
    std::vector<int64_t> eoff(ns + 1, 0);
    for (int64_t k = 0; k < ns; k++) {
        std::vector<int32_t> u;
        for (int64_t i = row0[k]; i < row0[k + 1]; i++)
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) u.push_back(col[e] - (int32_t)i);
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        auto it = dict.find(u);
        if (it == dict.end()) {
            it = dict.emplace(u, (int32_t)pats.size()).first;
            pats.push_back(u);
            if ((int64_t)pats.size() > std::max<int64_t>(64, ns / 8)) return false;  // unstructured
        }
        pid[k] = it->second;
        elems += (int64_t)((u.size() + L - 1) / L) * 64;
        eoff[k + 1] = elems;
    }
    if ((double)elems > 1.3 * (double)m.nnz) return false;  // too much padding
    std::vector<int32_t> poff(pats.size() + 1, 0), offs;
    for (size_t p = 0; p < pats.size(); p++) {
        offs.insert(offs.end(), pats[p].begin(), pats[p].end());
        poff[p + 1] = (int32_t)offs.size();
    }
    std::vector<double> val(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), m.val.get(), m.nnz * sizeof(double), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    std::vector<unsigned long long> tab;
    int vb = csr_value_table(m, tab);
    if (vb == 4) vb = 8;
    // operators with a value table keep the value-code SELL: its 16-B code units
    // with two rows per lane beat L lanes per row there (A_2 of the 256^3 cycle:
    // 56 vs 91 us), the dependent table gather is the chain either way
    if (vb) return false;
    std::vector<double> ev(elems, 0.0);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t k = 0; k < ns; k++) {
        const std::vector<int32_t> &u = pats[pid[k]];
        for (int64_t i = row0[k]; i < row0[k + 1]; i++) {
            const int r = (int)(i - row0[k]);
            size_t t = 0;
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
                const int32_t o = col[e] - (int32_t)i;
                while (u[t] != o) t++;
                ev[eoff[k] + (int64_t)(t / L) * 64 + r * L + t % L] = val[e];
            }
        }
    }
    m.sellp_vbits = vb;
    if (vb) {
        const int cb = vb / 8;
        std::vector<uint8_t> codes(elems * cb);
#pragma omp parallel for schedule(static)
        for (int64_t e = 0; e < elems; e++) {
            unsigned long long bits;
            std::memcpy(&bits, &ev[e], 8);
            const int c = (int)(std::lower_bound(tab.begin(), tab.end(), bits) - tab.begin());
            if (cb == 1) codes[e] = (uint8_t)c;
            else reinterpret_cast<uint16_t *>(codes.data())[e] = (uint16_t)c;
        }
        m.sellp_vals.resize(std::max<int64_t>(16, elems * cb));
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vals.get(), codes.data(), elems * cb, hipMemcpyHostToDevice, st));
        m.sellp_vtab.resize(tab.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vtab.get(), tab.data(), tab.size() * 8, hipMemcpyHostToDevice, st));
        m.sellp_ntab = (int64_t)tab.size();
    } else {
        m.sellp_vals.resize(std::max<int64_t>(16, elems * 8));
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vals.get(), ev.data(), elems * 8, hipMemcpyHostToDevice, st));
        m.sellp_ntab = 0;
    }
    m.sellp_eoff.resize(ns + 1);
    m.sellp_row0.resize(ns + 1);
    m.sellp_pid.resize(std::max<int64_t>(1, ns));
    m.sellp_poff.resize(poff.size());
    m.sellp_offs.resize(std::max<size_t>(1, offs.size()));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_eoff.get(), eoff.data(), (ns + 1) * 8, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_row0.get(), row0.data(), (ns + 1) * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_pid.get(), pid.data(), ns * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_poff.get(), poff.data(), poff.size() * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_offs.get(), offs.data(), offs.size() * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    m.sellp_slices = ns;
    m.sellp_elems = elems;
    m.sellp_L = L;
    m.sellp_seg_slc = seg_slc;
    m.sellp_meta_bytes = (int64_t)(16 * (ns + 1) + 4 * poff.size() + 4 * offs.size());
    return true;
}

void spmv_sellp(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
                int64_t seg) {
    const int64_t s0 = seg < 0 ? 0 : m.sellp_seg_slc[seg];
    const int64_t s1 = seg < 0 ? m.sellp_slices : m.sellp_seg_slc[seg + 1];
    if (s1 <= s0) return;
    SellpArgs a{m.sellp_vals.get(), m.sellp_eoff.get(), m.sellp_row0.get(), m.sellp_pid.get(), m.sellp_poff.get(),
                m.sellp_offs.get(), m.sellp_vtab.get(), (int32_t)s0, (int32_t)(s1 - s0), (int32_t)m.ncols,
                x, y, epi.b, epi.d, epi.dc, epi.dt};
    const dim3 grid((unsigned)ceil_div(s1 - s0, 4)), block(256);
#define FAMG_SELLP(L, VB)                                                                          \
    switch (mode) {                                                                                \
    case SPMV_SET: spmv_sellp_kernel<SPMV_SET, L, VB><<<grid, block, 0, s>>>(a); break;            \
    case SPMV_ADD: spmv_sellp_kernel<SPMV_ADD, L, VB><<<grid, block, 0, s>>>(a); break;            \
    case SPMV_RESID: spmv_sellp_kernel<SPMV_RESID, L, VB><<<grid, block, 0, s>>>(a); break;        \
    case SPMV_JACOBI: spmv_sellp_kernel<SPMV_JACOBI, L, VB><<<grid, block, 0, s>>>(a); break;      \
    default: fail(AMG_ERR_UNSUPPORTED, "pattern SELL: unsupported SpMV epilogue");                 \
    }
#define FAMG_SELLP_VB(L)                                                                           \
    if (m.sellp_vbits == 0) { FAMG_SELLP(L, 0) }                                                   \
    else if (m.sellp_vbits == 8) { FAMG_SELLP(L, 8) }                                              \
    else { FAMG_SELLP(L, 16) }
    switch (m.sellp_L) {
    case 2: FAMG_SELLP_VB(2) break;
    case 4: FAMG_SELLP_VB(4) break;
    case 8: FAMG_SELLP_VB(8) break;
    case 16: FAMG_SELLP_VB(16) break;
    case 32: FAMG_SELLP_VB(32) break;
    default: FAMG_SELLP_VB(64) break;
    }
#undef FAMG_SELLP_VB
#undef FAMG_SELLP
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
