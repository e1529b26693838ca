// sellp.hip -- pattern SELL: slices of structured operators whose columns are
// implicit.
//
// A slice is R = 64 / L consecutive rows, each row's steps dealt round-robin to
// its L lanes.  Step t of row r reads column base(r) + off[t], off[] the sorted
// union of the slice's column offsets; base(r) is r for a square matrix and the
// row's smallest column otherwise (the restriction R = P^T of a box hierarchy:
// every interior row the same 32 fine-node offsets around its box).  Slices share
// their offset list through a dictionary of patterns, so the matrix stream is the
// values alone: fp64, or 4/8-bit codes into a <= 256-entry table staged in LDS
// (the SELL-64 code tables, same bit patterns).  16-bit-code operators keep
// SELL-64: with the table gathered from L2 its two-rows-per-lane 16-B units
// measured faster (A_2 of the 256^3 cycle: 56 vs 91 us).
//
// Lane l = r L + q of a slice owns the steps t = s L + q, s = 0..S-1, S =
// ceil(w / L).  fp64: element (s, l) at s * 64 + l.  Codes: K = 32 / VB of a
// lane's consecutive steps share one 32-bit word at (s / K) * 64 + l, bits
// (s % K) * VB -- one coalesced dword per lane per K steps.  Padding steps (a row
// without entry at an offset, t >= w) hold +0.0 at a clamped in-range column.
//
// Summation order: lane q sums its steps ascending with fma, then the L partial
// sums are combined by a fixed butterfly -- deterministic, and for L = 1 on
// rows stored in ascending column order the oracle's order exactly (bitwise row
// sums); otherwise rounding-level differences covered by the tolerance-based
// parity tests.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>

#include "famg.hpp"

namespace famg {

struct SellpArgs {
    const char *vals;       // fp64 values or packed 4/8-bit codes
    const int64_t *eoff;    // per slice: first unit (double or dword)
    const int32_t *row0;    // per slice: first row (+1 sentinel)
    const int2 *pat;        // per slice: its offset pattern {start in offs, width}
    const int32_t *offs;    // concatenated sorted offset patterns
    const int32_t *rbase;   // per row: column base (nullptr: the row itself)
    const double *vtab;
    int32_t ntab, slice0, nslices, ncols, w2, spw;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
    double *y2;  // SETDF: y2 = d * y (the next level's first Jacobi step from zero)
};

template <int MODE> __device__ __forceinline__ double sellp_x(const SellpArgs &a, int c) { return a.x[c]; }

// fp64 values: U lane-steps, every load issued before the fmas
template <int MODE, int L, int U>
__device__ __forceinline__ void sellp_f64(const SellpArgs &a, int64_t e0, const int32_t *__restrict__ off, int w,
                                          int s0, int q, int base, int lane, double &acc) {
    double v[U], xx[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int t = (s0 + u) * L + q;
        const bool in = t < w;
        const int c = min(max(base + off[in ? t : 0], 0), a.ncols - 1);
        const double val = __builtin_nontemporal_load(reinterpret_cast<const double *>(a.vals) + e0 +
                                                      (int64_t)(s0 + u) * 64 + lane);
        v[u] = in ? val : 0.0;
        xx[u] = sellp_x<MODE>(a, c);
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc = fma(v[u], xx[u], acc);
}

// codes: W dwords = W K lane-steps; all W K x loads issued before the fmas
template <int MODE, int L, int VB, int W>
__device__ __forceinline__ void sellp_words(const SellpArgs &a, const double *stab, const uint32_t *wp, int k0,
                                            const int32_t *__restrict__ off, int w, int q, int base, double &acc) {
    constexpr int K = 32 / VB;
    uint32_t wd[W];
#pragma unroll
    for (int j = 0; j < W; j++) wd[j] = __builtin_nontemporal_load(wp + (int64_t)(k0 + j) * 64);
    double v[W * K], xx[W * K];
#pragma unroll
    for (int u = 0; u < W * K; u++) {
        const int t = (k0 * K + u) * L + q;
        const bool in = t < w;
        const int c = min(max(base + off[in ? t : 0], 0), a.ncols - 1);
        v[u] = stab[(wd[u / K] >> ((u % K) * VB)) & ((1u << VB) - 1)];
        // L = 1: t is the same on every lane, so padding steps skip their gather
        xx[u] = (L > 1 || in) ? sellp_x<MODE>(a, c) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < W * K; u++) acc = fma(v[u], xx[u], acc);
}

template <int MODE, int L, int VB>
__device__ __forceinline__ void sellp_slice(const SellpArgs &a, const double *stab, int sl) {
    const int s = a.slice0 + sl;
    const int lane = threadIdx.x & 63;
    const int r = lane / L, q = lane % L;
    const int row = a.row0[s] + r;
    const bool live = row < a.row0[s + 1];
    const int rowc = live ? row : a.row0[s];
    const int base = a.rbase ? a.rbase[rowc] : rowc;
    double br = 0.0, xr = 0.0, dr = 0.0, yr = 0.0;
    if (live && q == 0) {  // epilogue operands first
        if constexpr (MODE == SPMV_RESID) br = a.b[row];
        if constexpr (MODE == SPMV_ADD) yr = a.y[row];
        if constexpr (MODE == SPMV_ADD0) yr = (a.dc ? a.dt[a.dc[row]] : a.d[row]) * a.b[row];
        if constexpr (MODE == SPMV_JACOBI) {
            xr = a.x[row];
            br = a.b[row];
            dr = a.dc ? a.dt[a.dc[row]] : a.d[row];
        }
        if constexpr (MODE == SPMV_SETDF) dr = a.dc ? a.dt[a.dc[row]] : a.d[row];
    }
    const int2 pw = a.pat[s];
    const int32_t *off = a.offs + pw.x;
    const int w = pw.y;
    const int S = (w + L - 1) / L;
    const int64_t e0 = a.eoff[s];
    double acc = 0.0;
    if constexpr (VB == 0) {
        int s0 = 0;
        if (a.w2)  // A/B (FAMG_SELLP_W1=1: groups of 4): groups of 8 lane-steps
            for (; s0 + 8 <= S; s0 += 8) sellp_f64<MODE, L, 8>(a, e0, off, w, s0, q, base, lane, acc);
        for (; s0 + 4 <= S; s0 += 4) sellp_f64<MODE, L, 4>(a, e0, off, w, s0, q, base, lane, acc);
        switch (S - s0) {
        case 1: sellp_f64<MODE, L, 1>(a, e0, off, w, s0, q, base, lane, acc); break;
        case 2: sellp_f64<MODE, L, 2>(a, e0, off, w, s0, q, base, lane, acc); break;
        case 3: sellp_f64<MODE, L, 3>(a, e0, off, w, s0, q, base, lane, acc); break;
        default: break;
        }
    } else {
        constexpr int K = 32 / VB;
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(a.vals) + e0 + lane;
        const int nw = (S + K - 1) / K;
        int k = 0;
        if (a.w2) for (; k + 2 <= nw; k += 2) sellp_words<MODE, L, VB, 2>(a, stab, wp, k, off, w, q, base, acc);
        for (; k < nw; k++) sellp_words<MODE, L, VB, 1>(a, stab, wp, k, off, w, q, base, acc);
    }
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    if (live && q == 0) {
        if constexpr (MODE == SPMV_SET) a.y[row] = acc;
        else if constexpr (MODE == SPMV_SETDF) {
            a.y[row] = acc;
            a.y2[row] = dr * acc;  // vec_mul(_coded)'s product
        } else if constexpr (MODE == SPMV_ADD || MODE == SPMV_ADD0) a.y[row] = yr + acc;
        else if constexpr (MODE == SPMV_RESID) a.y[row] = br - acc;
        else a.y[row] = xr + dr * (br - acc);  // JACOBI
    }
}

// Each wave takes a.spw consecutive slices (contiguous per XCD through the
// block remap).
template <int MODE, int L, int VB>
__global__ __launch_bounds__(256) void spmv_sellp_kernel(SellpArgs a) {
    __shared__ double stab[VB ? 256 : 1];
    if constexpr (VB != 0) {
        for (int i = threadIdx.x; i < a.ntab; i += 256) stab[i] = a.vtab[i];
        __syncthreads();
    }
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int wv = __builtin_amdgcn_readfirstlane(blk * 4 + (int)(threadIdx.x >> 6));
    const int s0 = wv * a.spw, s1 = min(s0 + a.spw, a.nslices);
    for (int sl = s0; sl < s1; sl++) sellp_slice<MODE, L, VB>(a, stab, sl);
}

static bool sellp_disabled() {
    static const bool off = [] {
        const char *e = getenv("FAMG_NO_SELLP");
        return e && e[0] == '1';
    }();
    return off;
}

void sellp_release(GpuCsr &m) {
    m.sellp_vals.release();
    m.sellp_eoff.release();
    m.sellp_row0.release();
    m.sellp_pat.release();
    m.sellp_offs.release();
    m.sellp_rbase.release();
    m.sellp_vtab.release();
    m.sellp_slices = m.sellp_elems = m.sellp_ntab = m.sellp_meta_bytes = m.sellp_stream = 0;
    m.sellp_L = 0;
    m.sellp_vbits = 0;
    m.sellp_seg_slc.clear();
}

// Builds the pattern-SELL storage when the rows of every slice share a small
// set of offset patterns (a structured operator): fp64-valued operators whose
// rows average >= 48 entries (then L >= 2 lanes per row); 4/8-bit-coded
// operators when the pattern stream is <= 0.5 of other_bytes (the storage
// finalize chose).  True if built.
bool build_sellp(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes) {
    sellp_release(m);
    if (g_spmv_format_policy != 0 || sellp_disabled() || m.no_sellp || m.nrows < 1024 || m.nnz == 0 ||
        m.ncols < 2)
        return false;
    const int64_t n = m.nrows;
    const bool square = m.nrows == m.ncols;
    std::vector<unsigned long long> tab;
    int vb = csr_value_table(m, tab);
    if (vb == 16) return false;  // SELL-64 16-bit codes (see the header)
    const double avg = (double)m.nnz / (double)n;
    if (vb == 0 && m.nnz < 48 * n) return false;
    // coded rows need >= 16 entries: one lane per short row plus its column base
    // cost more than the bytes save (P_0: 4-8 entries per row, 124 -> 131-155 us
    // on the 7-pt and 153 -> 167 us on the 27-pt cycle; R_0, 32-64 entries:
    // 83 -> 64 and 137 -> 91 us)
    if (vb != 0 && m.nnz < 16 * n) return false;
    // lanes per row: enough waves to fill the chip (>= 32K), >= 8 steps per lane
    int L = 1;
    while (L < 64 && (n * L) / 64 < 32768 && avg / (2 * L) >= 8) L *= 2;
    if (vb == 0 && L < 2) return false;
    const int R = 64 / L;
    const int K = vb ? 32 / vb : 1;
    hipStream_t st = m.ctx->stream;
    std::vector<int32_t> col(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), m.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    // column base per row: the row itself (square) or its smallest column
    std::vector<int32_t> base(n);
    // (columns need not ascend within a row: a distributed level's [owned | ghost] numbering)
    for (int64_t i = 0; i < n; i++) {
        int32_t b = square ? (int32_t)i : INT32_MAX;
        if (!square)
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) b = std::min(b, col[e]);
        base[i] = b == INT32_MAX ? 0 : b;
    }
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
    std::vector<int64_t> eoff(ns + 1, 0);  // units: doubles (fp64) or dwords (codes)
    int64_t elems = 0;
    for (int64_t k = 0; k < ns; k++) {
        std::vector<int32_t> u;
        for (int64_t i = row0[k]; i < row0[k + 1]; i++)
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) u.push_back(col[e] - base[i]);
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        if (u.empty()) u.push_back(0);
        auto it = dict.find(u);
        if (it == dict.end()) {
            it = dict.emplace(u, (int32_t)pats.size()).first;
            pats.push_back(u);
            if ((int64_t)pats.size() > std::max<int64_t>(64, ns / 8)) return false;  // unstructured
        }
        pid[k] = it->second;
        const int64_t S = ((int64_t)u.size() + L - 1) / L;
        eoff[k + 1] = eoff[k] + (vb ? (S + K - 1) / K : S) * 64;
        elems += S * 64;  // pattern slots (code words may hold a few more)
    }
    if (vb == 0 && (double)elems > 1.3 * (double)m.nnz) return false;  // too much padding (codes: bytes below)
    std::vector<int32_t> poff(pats.size() + 1, 0), offs;
    for (size_t p = 0; p < pats.size(); p++) {
        offs.insert(offs.end(), pats[p].begin(), pats[p].end());
        poff[p + 1] = (int32_t)offs.size();
    }
    const int64_t units = eoff[ns];
    const int64_t meta = (int64_t)(20 * (ns + 1) + 4 * offs.size()) + (square ? 0 : 4 * n);
    const int64_t stream = units * (vb ? 4 : 8) + meta + 8 * (int64_t)tab.size();
    // codes: at most half the bytes of the storage finalize chose (P_0 of the 256^3
    // cycle, 4 entries per row, streams 0.67 of its SELL-64 bytes but ran 131-155
    // vs 124 us: the per-row base and one row per lane cost what the bytes save)
    if (vb && (double)stream > 0.5 * (double)other_bytes) return false;
    std::vector<double> val(m.nnz);
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), m.val.get(), m.nnz * sizeof(double), hipMemcpyDeviceToHost, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    std::vector<double> fv;
    std::vector<uint32_t> words;
    int zero_code = 0;
    if (vb) {
        zero_code = (int)(std::lower_bound(tab.begin(), tab.end(), 0ull) - tab.begin());
        uint32_t zw = 0;
        for (int u = 0; u < 32 / vb; u++) zw |= (uint32_t)zero_code << (u * vb);
        words.assign(eoff[ns], zw);
    } else {
        fv.assign(units, 0.0);
    }
    const int KK = vb ? 32 / vb : 1;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t k = 0; k < ns; k++) {
        const std::vector<int32_t> &u = pats[pid[k]];
        for (int64_t i = row0[k]; i < row0[k + 1]; i++) {
            const int r = (int)(i - row0[k]);
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
                const int32_t o = col[e] - base[i];
                const size_t t = (size_t)(std::lower_bound(u.begin(), u.end(), o) - u.begin());
                const int64_t s = (int64_t)(t / L), lane = (int64_t)r * L + (int64_t)(t % L);
                if (vb == 0) {
                    fv[eoff[k] + s * 64 + lane] = val[e];
                } else {
                    unsigned long long bits;
                    std::memcpy(&bits, &val[e], 8);
                    const uint32_t c = (uint32_t)(std::lower_bound(tab.begin(), tab.end(), bits) - tab.begin());
                    uint32_t &wd = words[eoff[k] + (s / KK) * 64 + lane];
                    const int sh = (int)(s % KK) * vb;
                    wd = (wd & ~(((1u << vb) - 1) << sh)) | (c << sh);
                }
            }
        }
    }
    m.sellp_vbits = vb;
    if (vb) {
        m.sellp_vals.resize(std::max<int64_t>(16, (int64_t)words.size() * 4));
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vals.get(), words.data(), words.size() * 4, hipMemcpyHostToDevice, st));
        m.sellp_vtab.resize(tab.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vtab.get(), tab.data(), tab.size() * 8, hipMemcpyHostToDevice, st));
        m.sellp_ntab = (int64_t)tab.size();
    } else {
        m.sellp_vals.resize(std::max<int64_t>(16, units * 8));
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_vals.get(), fv.data(), units * 8, hipMemcpyHostToDevice, st));
        m.sellp_ntab = 0;
    }
    if (!square) {
        m.sellp_rbase.resize(n);
        FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_rbase.get(), base.data(), n * 4, hipMemcpyHostToDevice, st));
    }
    m.sellp_eoff.resize(ns + 1);
    m.sellp_row0.resize(ns + 1);
    std::vector<int32_t> pat(2 * std::max<int64_t>(1, ns), 0);
    for (int64_t k = 0; k < ns; k++) {
        pat[2 * k] = poff[pid[k]];
        pat[2 * k + 1] = poff[pid[k] + 1] - poff[pid[k]];
    }
    m.sellp_pat.resize(pat.size());
    m.sellp_offs.resize(std::max<size_t>(1, offs.size()));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_eoff.get(), eoff.data(), (ns + 1) * 8, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_row0.get(), row0.data(), (ns + 1) * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_pat.get(), pat.data(), pat.size() * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.sellp_offs.get(), offs.data(), offs.size() * 4, hipMemcpyHostToDevice, st));
    FAMG_CHECK_HIP(hipStreamSynchronize(st));
    m.sellp_slices = ns;
    m.sellp_elems = vb ? eoff[ns] * (32 / vb) : units;
    m.sellp_L = L;
    m.sellp_seg_slc = seg_slc;
    m.sellp_meta_bytes = meta;
    m.sellp_stream = (vb ? eoff[ns] * 4 : units * 8) + meta + 8 * m.sellp_ntab;
    return true;
}

// two code words per step group (A/B switch FAMG_SELLP_W1=1: one)
static int sellp_w2_enabled() {
    static const int on = [] {
        const char *e = getenv("FAMG_SELLP_W1");
        return (e && e[0] == '1') ? 0 : 1;
    }();
    return on;
}

// slices per wave (A/B switch FAMG_SELLP_SPW=n, default 1)
static int sellp_spw() {
    static const int v = [] {
        const char *e = getenv("FAMG_SELLP_SPW");
        const int k = e ? atoi(e) : 1;
        return k > 0 ? k : 1;
    }();
    return v;
}

void spmv_sellp(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
                int64_t seg) {
    const int64_t s0 = seg < 0 ? 0 : m.sellp_seg_slc[seg];
    const int64_t s1 = seg < 0 ? m.sellp_slices : m.sellp_seg_slc[seg + 1];
    if (s1 <= s0) return;
    SellpArgs a{m.sellp_vals.get(), m.sellp_eoff.get(), m.sellp_row0.get(),
                reinterpret_cast<const int2 *>(m.sellp_pat.get()), m.sellp_offs.get(), m.sellp_rbase.get(), m.sellp_vtab.get(), (int32_t)m.sellp_ntab,
                (int32_t)s0, (int32_t)(s1 - s0), (int32_t)m.ncols, sellp_w2_enabled(), sellp_spw(), x, y, epi.b, epi.d, epi.dc, epi.dt,
                epi.y2};
    FAMG_REQUIRE(mode != SPMV_SETDF || (epi.y2 && (epi.d || epi.dc)), AMG_ERR_INVALID, "SETDF needs y2 and d");
    const dim3 grid((unsigned)ceil_div(s1 - s0, 4 * (int64_t)a.spw)), block(256);
#define FAMG_SELLP(L, VB)                                                                          \
    switch (mode) {                                                                                \
    case SPMV_SET: spmv_sellp_kernel<SPMV_SET, L, VB><<<grid, block, 0, s>>>(a); break;            \
    case SPMV_ADD: spmv_sellp_kernel<SPMV_ADD, L, VB><<<grid, block, 0, s>>>(a); break;            \
    case SPMV_RESID: spmv_sellp_kernel<SPMV_RESID, L, VB><<<grid, block, 0, s>>>(a); break;        \
    case SPMV_JACOBI: spmv_sellp_kernel<SPMV_JACOBI, L, VB><<<grid, block, 0, s>>>(a); break;      \
    case SPMV_ADD0: spmv_sellp_kernel<SPMV_ADD0, L, VB><<<grid, block, 0, s>>>(a); break;          \
    case SPMV_SETDF: spmv_sellp_kernel<SPMV_SETDF, L, VB><<<grid, block, 0, s>>>(a); break;        \
    default: fail(AMG_ERR_UNSUPPORTED, "pattern SELL: unsupported SpMV epilogue");                 \
    }
#define FAMG_SELLP_VB(L)                                                                           \
    if (m.sellp_vbits == 0) { FAMG_SELLP(L, 0) }                                                   \
    else if (m.sellp_vbits == 4) { FAMG_SELLP(L, 4) }                                              \
    else { FAMG_SELLP(L, 8) }
    switch (m.sellp_L) {
    case 1: FAMG_SELLP_VB(1) break;
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
