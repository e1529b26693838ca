// famg.hpp -- host-side object model of the MI355X AMG library.
//
// The classes mirror the reference's operator surface (faer matrix_free
// LinOp / Precond / BiPrecond as used by aujxn/faer-amg):
//   LinOp            <- faer::matrix_free::LinOp<f64>        (trait object)
//   CsrOp            <- SparseMatOp / ParSpmmOp / SparseRowMat (core.rs, par_spmm.rs)
//   DiagOp           <- Diag<f64> from new_jacobi/new_l1/new_l2 (smoothers.rs:43-86)
//   SgsOp            <- SmootherKind::SymGaussSeidel (smoothers.rs:20, unimplemented there)
//   CoarseCholOp     <- SparseCholeskySolve (coarse_solvers.rs:164-276)
//   MultigridOp      <- Multigrid (preconditioners/multigrid.rs:171-518)
// All operator data lives in HBM; apply() works on device pointers and is
// asynchronous on the context stream.
#pragma once

#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace famg {

// Workgroup b of nb -> the b-th of a contiguous range per XCD (consecutive
// workgroups round-robin over the 8 XCDs, each with its own L2): each XCD then
// walks a contiguous slab of rows and keeps its x window in its L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, idx = b >> 3;
    return x * q + min(x, r) + idx;
}

// q / d for 0 <= q < 2^14 through a float reciprocal r = 1.0f / d: (q + 0.5) / d
// lies at least 0.5 / d from an integer, far beyond the float error, for the
// window and tile extents the staging loops divide by.  fdiv_exact checks every
// q < n on the host before a kernel relies on it (memoised per (n, d) in a
// per-thread table: the eager launch paths of the loopback ranks call it
// without a lock).
__device__ __forceinline__ int fdiv_rcp(int q, float r) { return (int)(((float)q + 0.5f) * r); }
inline bool fdiv_exact(int n, int d, float r) {
    thread_local std::vector<std::pair<int, int>> ok;
    for (const auto &e : ok)
        if (e.first >= n && e.second == d) return true;
    for (int q = 0; q < n; q++)
        if ((int)(((float)q + 0.5f) * r) != q / d) return false;
    ok.push_back({n, d});
    return true;
}

// ------------------------------------------------------------------ CSR data

// Plane layout of a rank-local vector of a distributed grid level (dist.hip,
// DESIGN.md 6): the rank owns planes [z0, z0 + nz) of an nx x ny x gz grid
// (local entries [0, nz * pl)), then its ghost planes -- gl whole planes below z0,
// then gh above z0 + nz.  Local plane z in [-gl, nz + gh) starts at entry
// z * pl + (z < 0 ? nz * pl + gl * pl : z >= nz ? gl * pl : 0).
// Off (nx == 0) for single-GPU matrices; a redundant (all-gathered) level is
// the frame with z0 = 0, nz = gz and no ghosts.
struct SlabFrame {
    int64_t nx = 0, ny = 0, gz = 0;  // the global grid
    int64_t z0 = 0, nz = 0;          // owned planes
    int64_t gl = 0, gh = 0;          // ghost planes below / above
    bool on() const { return nx > 0; }
    int64_t pl() const { return nx * ny; }
    int64_t n_own() const { return nz * nx * ny; }
    int64_t add_lo() const { return (nz + gl) * nx * ny; }  // added to z * pl for z < 0
    int64_t add_hi() const { return gl * nx * ny; }         // ... for z >= nz
    // global grid plane of a local entry (ghosts included)
    int64_t plane_of(int64_t c) const {
        const int64_t p = pl(), own = n_own();
        if (c < own) return z0 + c / p;
        const int64_t g = c - own;
        return g < gl * p ? z0 - gl + g / p : z0 + nz + (g - gl * p) / p;
    }
    int64_t in_plane(int64_t c) const {
        const int64_t p = pl(), own = n_own();
        return c < own ? c % p : (c - own) % p;
    }
};

// A CSR matrix resident on the device.  rp64 (int64 row pointers) always
// exists and is what setup kernels (SpGEMM, transpose, extraction) read;
// rp32 + the stream schedule exist when nnz < 2^31 and are what SpMV reads
// (12 B per entry + 4 B per row of index/value traffic).
struct GpuCsr {
    Ctx *ctx = nullptr;
    int64_t nrows = 0, ncols = 0, nnz = 0;
    DevBuf<int64_t> rp64;
    DevBuf<int32_t> rp32;
    DevBuf<int32_t> col;   // padded by 4 entries (16-B vector loads)
    DevBuf<double> val;    // padded by 2 entries
    DevBuf<int32_t> sched; // stream-SpMV row blocks: nblocks+1 row starts
    int64_t nblocks = 0;
    // Row segments (SGS colors, halo boundary/interior): [seg_rows[g], seg_rows[g+1]).
    // Schedule blocks and SELL slices never straddle a segment.
    std::vector<int64_t> seg_rows, seg_blk, seg_slc;
    // SELL-64 copy with compressed column indices (spmv.hip, "SELL storage"):
    // slice s holds rows [sell_row0[s], sell_row0[s+1]) (<= 64), one lane per
    // row, sell_soff[s+1]-sell_soff[s] entry steps; sell_desc[s] = byte offset/128
    // of its block in sell_data | column mode << 30; sell_base = one int32 per step.
    DevBuf<int32_t> sell_row0;
    DevBuf<int32_t> sell_soff;
    DevBuf<uint32_t> sell_desc;
    DevBuf<int32_t> sell_base;
    DevBuf<char> sell_data;
    int64_t nslices = 0, sell_steps = 0, sell_bytes = 0;
    int64_t sell_mode_slices[3] = {0, 0, 0};  // slices per column mode (implicit, u16, i32)
    bool sell_paired = true;  // step-pair layout (16-B value loads); false: one step per 512-B row
    bool sell_short = false;  // coded slices of <= 4 steps in equal pairs (spmv_sell_short_kernel)
    // value codes (spmv.hip "value codes"): 0 = fp64 values, else 4/8/16-bit codes
    // into sell_vtab (sell_ntab distinct bit patterns, ascending)
    int sell_vbits = 0;
    int64_t sell_ntab = 0;
    DevBuf<double> sell_vtab;
    // DIA codes (spmv.hip "DIA codes"): dia_cw words of codes per row for the
    // dia_k diagonals dia_off (ascending); value table = sell_vtab
    DevBuf<uint32_t> dia_codes;
    DevBuf<double> dia_vtab;
    int64_t dia_ntab = 0;
    int dia_k = 0, dia_cw = 0, dia_vbits = 0;
    int dia_pat = 0;  // > 32 diagonals: the run pattern (spmv_dia_pat_kernel)
    // 7- or 27-point DIA operator whose every row is the interior stencil truncated
    // at the grid faces (dia_constant): the kernels read no codes
    bool dia_cst = false;
    int dia_cst_n[3] = {0, 0, 0};
    double dia_cst_v[27] = {0};
    std::vector<int> dia_off;
    // DIA row range: the whole matrix (kernel == DIA) or one row segment
    // (dia_seg, e.g. the halo interior of a distributed level) beside SELL
    int64_t dia_r0 = 0, dia_r1 = 0, dia_seg = 0;
    // set when the DIA codes describe a color-permuted SGS copy: stored row p
    // is original row dia_rowid[p] (device array owned by the SgsOp)
    const int32_t *dia_rowid = nullptr;
    // wave-per-row storage compression: 8/16-bit value codes (vec_codes, table
    // sell_vtab) and 16-bit column offsets from the row (vec_off)
    DevBuf<uint8_t> vec_codes;
    DevBuf<int16_t> vec_off;
    int vec_vbits = 0;
    bool vec_o16 = false;
    int vec_wpr = 1;  // waves per row, chosen once for the whole matrix (flag FLAG_VEC_WPR overrides)
    // 3x3 block storage (bsr.hip): node-row slices, one 4864-B unit per block step
    DevBuf<char> bsr_data;
    DevBuf<int32_t> bsr_row0, bsr_soff;
    int64_t bsr_slices = 0, bsr_steps = 0, bsr_maxw = 0;
    std::vector<int64_t> bsr_seg_slc;
    bool no_bsr = false;  // e.g. a color-permuted SGS copy
    bool bsr_pin = false;  // a renumbered copy of a 3x3-block matrix: take the block storage whenever it builds
    int8_t kind_pin = -1;  // a renumbered copy: 0 one-lane storages (SELL / x-staged) whenever they build, 1 wave-per-row, 2 CSR-stream
    // pattern SELL with L lanes per row (sellp.hip): values / codes only, columns
    // from per-slice offset patterns
    DevBuf<char> sellp_vals;
    DevBuf<int64_t> sellp_eoff;
    DevBuf<int32_t> sellp_row0, sellp_pat, sellp_offs;  // pat: {offs start, width} per slice
    DevBuf<int32_t> sellp_rbase;  // per-row column base (rectangular matrices)
    DevBuf<double> sellp_vtab;
    int64_t sellp_slices = 0, sellp_elems = 0, sellp_ntab = 0, sellp_meta_bytes = 0, sellp_stream = 0;
    bool no_sellp = false;  // e.g. a color-permuted SGS copy (swept in SGS mode)
    int sellp_L = 0, sellp_vbits = 0;
    std::vector<int64_t> sellp_seg_slc;
    // stencil-class storage (scs.hip): one 8/16-bit class id per row, a
    // dictionary of class stencils over the union of the rows' offsets
    DevBuf<char> scs_cls;
    DevBuf<double> scs_dict;
    DevBuf<int32_t> scs_offs;
    int64_t scs_k = 0, scs_nclass = 0;
    int64_t scs_kr = 0;  // offsets before the padding to a multiple of 8 (the x-staged walk stops there)
    int64_t scs_seg = -1;  // >= 0: only this row segment (a distributed level's halo interior) beside SELL
    int scs_ib = 0;
    bool scs_lanes = false;  // one row per wave (few long rows: spmv_scs_lanes_kernel)
    // x-staged stencil classes on a 3-D grid (scs.hip, spmv_xscs_kernel): per tile
    // of tx x ty x tz grid points its x window (tile + halo rx/ry/rz) in LDS;
    // xscs_lo[k] = the window offset of stencil offset k
    bool xscs = false;
    int xscs_t[3] = {0, 0, 0}, xscs_r[3] = {0, 0, 0};
    int xscs_ws = 0;  // LDS row stride of the window (>= wx; padded against bank conflicts)
    int xscs_tile_src = 0;  // how the tile was chosen: TuneSource (tuning.hpp)
    bool xscs_fdiv = false;  // the tile's float-reciprocal divisions checked exact (xscs_set_tile)
    DevBuf<int32_t> xscs_lo;
    std::vector<int> xscs_steps;  // (dx, dy, dz) of each of the scs_k offsets
    // grid-transfer classes (gtc.hip) for R/P of a 2x2x2-box hierarchy: an overlay
    // on the finalized storage used for the modes it supports (gtc_supports)
    bool gtc_on = false, gtc_r = false;
    bool gtc_tried = false;  // gtc_attach ran since the last finalize (attach_box_transfers retries nothing)
    DevBuf<uint8_t> gtc_cls;
    DevBuf<uint16_t> gtc_dict;  // nclass x ke entries: value index << 8 | step slot
    DevBuf<double> gtc_vtab;    // the distinct values (<= 256)
    int gtc_ke = 0, gtc_nce = 0, gtc_ntab = 0, gtc_nclass = 0;
    // R: per class the first entry of each fine-plane group dz = -1, 0, 1, 2 and the
    // real entry count (5 bytes; the marching fused restriction of fine.hip)
    DevBuf<uint8_t> gtc_kdz;
    // R: per class its value at each of the 32 slots (dz, dy, dx) a 2 x 2 x 2 box
    // smoothed by the 7-point stencil reaches, +0.0 where the class has no entry
    // (fine.hip k_fine_rr); empty when some class has an entry outside them
    DevBuf<double> gtc_wt;
    int64_t gtc_fg[3] = {0, 0, 0}, gtc_cg[3] = {0, 0, 0};
    // wide grid-transfer classes (gtx.hip): 16-bit class per row, dictionary of
    // (window offset, fp64 value) entries in global memory -- every box level
    bool gtx_on = false, gtx_r = false, gtx_tried = false;
    DevBuf<uint16_t> gtx_cls;
    DevBuf<int32_t> gtx_dptr, gtx_dlen, gtx_doff;
    DevBuf<double> gtx_dval;
    int64_t gtx_nclass = 0, gtx_nent = 0;
    int gtx_tile[3] = {0, 0, 0}, gtx_win[3] = {0, 0, 0}, gtx_lo[3] = {0, 0, 0};
    int64_t gtx_fg[3] = {0, 0, 0}, gtx_cg[3] = {0, 0, 0};
    bool gtx_fdiv = false;  // the window's float-reciprocal divisions checked exact (at build)
    // grid hint: the rows are the points of an nx x ny x nz grid, x fastest (0 = none);
    // set by the stencil generators, the box hierarchy and amg_csr_set_grid
    // (grid_src 1), else inferred at finalize from the stencil offsets (grid_src 2)
    int64_t grid[3] = {0, 0, 0};
    int grid_src = 0;
    // rank-local matrix of a distributed grid level (dist.hip): its rows are the
    // owned planes of rframe, its columns the local vector of cframe.  The
    // x-staged classes and grid-transfer classes then stage ghost planes through
    // the frame, and their launches split into interior / boundary z-tile ranges
    // (segments 1 / 0, 2) so the interior runs while the halo is in flight.
    SlabFrame rframe, cframe;
    // x-staged SELL (xsell.hip): per group of 4096 rows the x chunks staged in LDS,
    // per slice fp64 values + 16-bit LDS indices (or 32-bit columns: escape slices)
    DevBuf<char> xs_data;
    DevBuf<uint32_t> xs_desc;
    DevBuf<int32_t> xs_soff, xs_coff, xs_chunks;
    int64_t xs_groups = 0, xs_bytes = 0, xs_steps = 0, xs_chunk_total = 0, xs_escape_slices = 0;
    int64_t xs_maxw = 0;  // widest slice (the burst kernel's batch: 7 or 8 steps)
    // a renumbered copy (reorder.hip): rows in a new order, each row's entries in
    // the original's stored order with renamed columns -- storages that reorder a
    // row's entries (DIA, stencil / grid-transfer classes, pattern and aligned SELL)
    // are not built, so every row sum stays the original's; col_orig = new column ->
    // original column (the 3x3-block build merges a node's rows by original column)
    bool order_fixed = false;
    std::vector<int32_t> col_orig;
    int kernel = 0;  // SpmvKernel chosen at finalize
    bool spmv_ready() const { return rp32.get() != nullptr && sched.get() != nullptr; }
    bool has_sell() const { return sell_desc.get() != nullptr; }
    bool has_dia() const { return dia_codes.get() != nullptr; }
    bool has_bsr() const { return bsr_data.get() != nullptr; }
    bool has_sellp() const { return sellp_vals.get() != nullptr; }
    bool has_scs() const { return scs_cls.get() != nullptr; }
    bool has_xs() const { return xs_data.get() != nullptr; }
    int64_t index_bytes() const { return 12 * nnz + 4 * (nrows + 1); }
    // matrix bytes one SpMV streams with the chosen kernel (data + metadata)
    int64_t stream_bytes() const {
        if (kernel == 3) return dia_cst ? 8 * (int64_t)dia_k : 4 * dia_cw * nrows + 8 * dia_ntab;  // constant: no codes
        if (kernel == 4) return bsr_steps * (64 * 76) + 8 * (bsr_slices + 1);
        if (kernel == 5) return sellp_stream;
        if (kernel == 6) return scs_ib * nrows + 8 * scs_k * scs_nclass + 4 * scs_k;
        if (kernel == 7) return xs_bytes + 8 * (int64_t)(xs_desc.size() + 1) + 4 * xs_chunk_total + 4 * (xs_groups + 1);
        if (kernel == 2)
            return nnz * ((vec_vbits ? vec_vbits / 8 : 8) + (vec_o16 ? 2 : 4)) + 4 * (nrows + 1) + 8 * sell_ntab;
        return kernel == 1 ? sell_bytes + 12 * (nslices + 1) + 4 * sell_steps + 8 * sell_ntab : index_bytes();
    }
};

// Grid dims (nx, ny, nz) of a square operator of n rows whose stencil has the
// offsets offs (col - row over some rows); false if no grid explains them.
bool grid_from_offsets(const std::vector<int64_t> &offs, int64_t n, int64_t *g);
// R and P of a 2x2x2-box level as grid-transfer classes when the fine and coarse
// operators carry grid hints of that relation (Multigrid::add_level)
void attach_box_transfers(const GpuCsr &Af, const GpuCsr &Ac, GpuCsr &R, GpuCsr &P);
// Allocate a CSR with the given shape/nnz (arrays uninitialised).
void csr_alloc(GpuCsr &m, Ctx *ctx, int64_t nrows, int64_t ncols, int64_t nnz);
// Device copy of the CSR arrays (rp64/col/val) of src into dst; dst is not
// finalized (call csr_finalize for its SpMV storage).
void csr_clone(const GpuCsr &src, GpuCsr &dst);
// Build rp32 (if nnz < 2^31), the stream schedule, the SELL-64 copy for short
// regular rows, and pick the SpMV kernel; `segments` (row bounds, first 0, last
// nrows) keeps blocks/slices inside segments.  Host pass over the row pointers
// (setup only).  Must be called again after values change in place.
void csr_finalize(GpuCsr &m, const std::vector<int64_t> *segments = nullptr);
// Format policy (process-wide, for matrices finalized afterwards):
// 0 auto, 1 CSR-stream only, 2 SELL whenever rows <= 256, 3 vector (no SELL)
extern int g_spmv_format_policy;
// Value codes for SELL matrices finalized afterwards (1 = when <= 65536
// distinct values, 0 = always fp64 values)
extern int g_value_codes;
enum SpmvKernel : int {
    SPMV_KERNEL_STREAM = 0, SPMV_KERNEL_SELL = 1, SPMV_KERNEL_VECTOR = 2, SPMV_KERNEL_DIA = 3, SPMV_KERNEL_BSR = 4,
    SPMV_KERNEL_SELLP = 5, SPMV_KERNEL_SCS = 6, SPMV_KERNEL_XS = 7, SPMV_KERNEL_GTC = 8
};
// grid-transfer classes (gtc.hip): fg/cg the fine/coarse grids of a 2x2x2-box
// level; the row classes of P (fine rows) or R (coarse rows) as (slot, value)
// lists; gtc_attach builds the overlay storage (true if it applies)
bool gtc_classes(const GpuCsr &M, bool is_r, const int64_t *fg, const int64_t *cg, std::vector<uint8_t> &cls,
                 std::vector<std::vector<std::pair<uint8_t, double>>> &dict);
// which: 1 = R (coarse rows), 0 = P (fine rows), -1 = R if it has fewer rows than columns
bool gtc_attach(GpuCsr &m, const int64_t *fg, const int64_t *cg, int which = -1);
void gtc_release(GpuCsr &m);
// stencil-class storage for structured operators whose rows repeat up to a
// shift; true if built (scs.hip)
bool build_scs(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes);
void scs_release(GpuCsr &m);
// x-staged SELL for gather-heavy fp64 SELL matrices; true if built (xsell.hip)
bool build_xs(GpuCsr &m, const std::vector<int64_t> &rp);
void xs_release(GpuCsr &m);
void sellp_release(GpuCsr &m);
// pattern SELL (implicit columns from per-slice offset patterns) for structured
// operators; true if built (sellp.hip)
bool build_sellp(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes);
int csr_value_table(const GpuCsr &m, std::vector<unsigned long long> &tab);
// 3x3 block storage when the matrix is blocked and it streams fewer bytes than
// other_bytes; true if built (bsr.hip)
bool build_bsr(GpuCsr &m, const std::vector<int64_t> &rp, int64_t other_bytes);
void build_sell(GpuCsr &m, const std::vector<int64_t> &rp);
// DIA codes of a color-permuted SGS copy (diagonals col - rowid[p]); true if built
bool build_dia_sgs(GpuCsr &m, const int32_t *rowid);
void choose_kernel(GpuCsr &m);
// Host upload from usize-compatible arrays.
void csr_from_host(GpuCsr &m, Ctx *ctx, int64_t nrows, int64_t ncols, const int64_t *rowptr,
                   const int64_t *col, const double *val);
void csr_to_host(const GpuCsr &m, int64_t *rowptr, int64_t *col, double *val);
// Diagonal a_ii per row (device, n); throws if a diagonal entry is missing.
void csr_diagonal(const GpuCsr &m, double *d_out);
void csr_abs_row_sums(const GpuCsr &m, double *d_out);

// ------------------------------------------------------------------ kernels

enum SpmvMode : int {
    SPMV_SET = 0,    // y = A x
    SPMV_ADD = 1,    // y = y + A x
    SPMV_RESID = 2,  // y = b - A x
    SPMV_JACOBI = 3, // y = x + d (b - A x)   (x != y)
    SPMV_SGS = 4,    // e[perm p] = e[perm p] + d_p (b[perm p] - (A e)_p)
    // the zero-guess Jacobi step v = d*b folded into its consumers (never stored):
    SPMV_RESID0 = 5, // y = b - A (d*b)   (x == b; d gathered with x)
    SPMV_ADD0 = 6,   // y = d*b + A x
    // restriction that also takes the next level's first Jacobi step from zero:
    // y = A x, y2 = d*y (wide grid-transfer classes only, gtx.hip)
    SPMV_SETDF = 7
};

struct SpmvEpi {
    const double *b = nullptr;
    const double *d = nullptr;
    const int32_t *perm = nullptr;
    const uint8_t *dc = nullptr;  // JACOBI only: 8-bit codes of d into dt
    const double *dt = nullptr;
    double dk = 0.0;              // d when every entry is this one value (0: not constant)
    double *y2 = nullptr;         // SETDF: the second output d*y
};

// y = epilogue(A x) over all rows (seg < 0) or over row segment `seg`, with the
// kernel chosen for m at finalize (SELL-64 / vector / CSR-stream).
// Y = A X for k columns (column-major, leading dimensions ldx/ldy): SELL
// matrices stream once per 8 columns; bitwise equal to k SpMVs.
void spmm(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k, hipStream_t s);
// the same for DIA-code, stencil-class and 3x3-block storage; false if m has none of them
bool spmm_compressed(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k,
                     hipStream_t s);
void spmv(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
          hipStream_t s, int64_t seg = -1);
void spmv_bsr(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg);
void spmv_scs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg);
bool xs_supports(SpmvMode mode);
// Y = A X over k columns on x-staged SELL (xsell.hip); false for other storages
bool spmm_xs(const GpuCsr &m, const double *x, int64_t ldx, double *y, int64_t ldy, int64_t k, hipStream_t s);
// the constant 7-point DIA kernel with a one-value Jacobi diagonal takes m's
// JACOBI / RESID0 launches (spmv.hip: no codes read, d = epi.dk)
bool dia7_cst_dk(const GpuCsr &m, const SpmvEpi &epi);
// fine.hip: the folded correction v = d f + P v_c and one Jacobi step on a
// constant 7-point fine level as one marching kernel (out = the Jacobi result)
bool fine_interp_jacobi_ok(const GpuCsr &A, const GpuCsr &P, const SpmvEpi &epi);
void fine_interp_jacobi(const GpuCsr &A, const GpuCsr &P, const double *vc, const double *f, double dk, double *out,
                        hipStream_t s);
// the folded residual r = f - A (d f) and f_c = R r, d_c f_c (SETDF) as one marching kernel
// (epic: the coarse level's d and y2 = d_c f_c, as spmv's SETDF epilogue takes them)
bool fine_resid_restrict_ok(const GpuCsr &A, const GpuCsr &R, const SpmvEpi &epi, const SpmvEpi &epic);
void fine_resid_restrict(const GpuCsr &A, const GpuCsr &R, const double *f, double dk, double *fc,
                         const SpmvEpi &epic, hipStream_t s);
bool gtc_supports(const GpuCsr &m, SpmvMode mode);
// wide grid-transfer classes (gtx.hip); which as gtc_attach
bool gtx_attach(GpuCsr &m, const int64_t *fg, const int64_t *cg, int which = -1);
void gtx_release(GpuCsr &m);
bool gtx_supports(const GpuCsr &m, SpmvMode mode);
int gtx_mode();
void spmv_gtx(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg = -1);
// seg < 0: every tile; a rank-local matrix (rframe on) also takes segments 1
// (interior z-tiles: no ghost reads) and 0 / 2 (the tiles before / after)
void spmv_gtc(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg = -1);
void spmv_xs(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s);
void spmv_sellp(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
                int64_t seg);

// BLAS-1 (n-vectors, device pointers)
void vec_fill(double *x, double v, int64_t n, hipStream_t s);
void vec_copy(double *dst, const double *src, int64_t n, hipStream_t s);
void vec_sub(double *out, const double *a, const double *b, int64_t n, hipStream_t s);  // a-b
void vec_add_inplace(double *x, const double *y, int64_t n, hipStream_t s);           // x+=y
void vec_mul(double *out, const double *d, const double *a, int64_t n, hipStream_t s); // d*a
// out = dt[dc] * a (8-bit codes of the diagonal)
void vec_mul_coded(double *out, const uint8_t *dc, const double *dt, const double *a, int64_t n, hipStream_t s);
// 8-bit codes of v (<= 256 distinct values): returns the table size, 0 if none built
// dconst (optional): set to the value when v holds one distinct nonzero value, else 0
int64_t array_codes_u8(const double *v, int64_t n, Ctx &ctx, DevBuf<uint8_t> &code, DevBuf<double> &table,
                       double *dconst = nullptr);
void vec_axpy(double *y, double alpha, const double *x, int64_t n, hipStream_t s);      // y+=a x
void vec_xpay(double *y, double beta, const double *x, int64_t n, hipStream_t s);       // y=x+b y
void vec_scale(double *x, double alpha, int64_t n, hipStream_t s);                      // x*=a
// x = x + d*(x - r)   (StationaryIteration quirk step, smoothers.rs:153-156)
void vec_nn_step(double *x, const double *d, const double *r, int64_t n, hipStream_t s);
// Deterministic dot product; result left on device in *res (fixed reduction tree).
void vec_dot_dev(const double *x, const double *y, int64_t n, double *res, Ctx &ctx);
// the same with the caller's partial sums (VEC_DOT_PARTIALS doubles): callers that share
// a context across threads (loopback ranks) must not share the context's scratch
constexpr int VEC_DOT_PARTIALS = 1024;
void vec_dot_dev(const double *x, const double *y, int64_t n, double *res, double *partials, hipStream_t s);
double vec_dot(const double *x, const double *y, int64_t n, Ctx &ctx);  // syncs

// marker kernel for rocprofv3 traces (amg_trace_mark)
void trace_mark(Ctx &ctx, int32_t tag);

// dense row-major GEMV: out = M * x (M n x n)
void dense_gemv(const double *M, const double *x, double *out, int64_t n, hipStream_t s);
// RCM node order (new -> old) of the node graph of an n x n CSR, bs dofs per node (reorder.hip)
std::vector<int32_t> rcm_order(const std::vector<int64_t> &rp, const std::vector<int32_t> &col, int64_t n, int bs);

// exclusive scan of int64 counts (n entries) into out (n+1 entries); returns total
int64_t scan_counts(const int64_t *counts, int64_t *out, int64_t n, Ctx &ctx);

// sparse products / setup
// C = A B; finalize = false leaves C without SpMV storage (setup intermediates)
void spgemm(const GpuCsr &A, const GpuCsr &B, GpuCsr &C, bool finalize = true);
// S += P where P's pattern lies within S's (values only; S is not re-finalized)
void csr_add_into(GpuCsr &S, const GpuCsr &P);
void transpose(const GpuCsr &A, GpuCsr &T);
void smooth_interp_fixup(GpuCsr &S, const GpuCsr &P, const double *diag, double omega);
void gen_stencil(GpuCsr &m, Ctx *ctx, int64_t nx, int64_t ny, int64_t nz, const int *offs,
                 const double *coef, int nsten);
// random-coefficient 7-pt operator (edge weights 0.5 + U[0,1), Dirichlet
// diagonal), rows/columns permuted symmetrically (window < 0 none, 0 all rows,
// > 0 within consecutive windows of that many rows)
void gen_random_7pt(GpuCsr &m, Ctx *ctx, int64_t nx, int64_t ny, int64_t nz, uint64_t seed, int64_t window);

// ------------------------------------------------------------------ operators

enum class Kind : int {
    Csr = AMG_KIND_CSR,
    Diag = AMG_KIND_DIAG,
    Sgs = AMG_KIND_SGS,
    Coarse = AMG_KIND_COARSE,
    Multigrid = AMG_KIND_MULTIGRID,
    DistCsr = AMG_KIND_DIST_CSR,
    DistMultigrid = AMG_KIND_DIST_MULTIGRID,
    Composite = AMG_KIND_COMPOSITE,
    Block = AMG_KIND_BLOCK
};

struct LinOp : std::enable_shared_from_this<LinOp> {
    Ctx *ctx = nullptr;
    int64_t nrows = 0, ncols = 0;
    virtual ~LinOp() = default;
    virtual Kind kind() const = 0;
    // LinOp::apply -- out = M rhs (device, one column), out overwritten.
    virtual void apply(double *out, const double *rhs) = 0;
    // BiLinOp::transpose_apply -- symmetric operators reuse apply.
    virtual void transpose_apply(double *out, const double *rhs) { apply(out, rhs); }
    // Precond::apply_in_place -- default: copy to scratch, then apply.
    virtual void apply_in_place(double *rhs);
    virtual bool is_precond() const { return false; }

  protected:
    DevBuf<double> inplace_scratch_;
};
using LinOpPtr = std::shared_ptr<LinOp>;

struct CsrOp : LinOp {
    GpuCsr m;
    DevBuf<double> diag_;  // cached a_ii (lazy)
    std::shared_ptr<CsrOp> transpose_;  // lazy, for transpose_apply
    Kind kind() const override { return Kind::Csr; }
    void apply(double *out, const double *rhs) override;
    void transpose_apply(double *out, const double *rhs) override;
    const double *diagonal();
};
using CsrPtr = std::shared_ptr<CsrOp>;

struct DiagOp : LinOp {
    DevBuf<double> d;
    // 8-bit codes of d (built by the multigrid when d has <= 256 distinct
    // values; the V-cycle's Jacobi steps then read 1 B per row instead of 8)
    DevBuf<uint8_t> dcode;
    DevBuf<double> dtab;
    double dconst = 0.0;  // d when it is one value (set with the codes), else 0
    bool codes_tried = false;
    Kind kind() const override { return Kind::Diag; }
    bool is_precond() const override { return true; }
    void apply(double *out, const double *rhs) override;
    void apply_in_place(double *rhs) override;
};

struct SgsOp : LinOp {
    CsrPtr A;              // original operator
    GpuCsr Ap;             // rows grouped by color (columns in original numbering)
    DevBuf<int32_t> perm;  // permuted row p -> original row
    DevBuf<double> dinv;   // 1/a_ii at permuted rows
    std::vector<int64_t> color_ptr;   // rows of color c: [color_ptr[c], color_ptr[c+1]) = Ap segment c
    std::vector<int32_t> host_colors;
    int64_t ncolors = 0;
    DevBuf<double> e_;     // scratch correction
    const double *aii_ = nullptr;  // setup only: a_ii of a rectangular slice's rows
    // fused plane-parity sweeps on a 27-point grid operator (sgs27.hip)
    bool fused27 = false;
    bool const27 = false;  // every row the interior stencil truncated at the faces: no codes loaded
    int nx27 = 0, ny27 = 0, nz27 = 0;
    std::vector<uint32_t> icode27;  // interior row's code group (8 words, unused = ~0)
    std::vector<double> icoef27;    // and its 27 coefficients
    std::vector<uint32_t> fmask27;  // 6 x 8 words: code bits of the entries leaving each grid face
    DevBuf<double> fused_tmp, fused_zero;
    Kind kind() const override { return Kind::Sgs; }
    bool is_precond() const override { return true; }
    // e = SGS(r) from e = 0 (device pointers, e != r)
    void sweep(double *e, const double *r);
    // x <- x + SGS(b - A x), in place on x
    void sweep_x(double *x, const double *b);
    // e_i = dinv_i r_i on the rows of color 0 (the first forward color from e = 0)
    void first_color(double *e, const double *r);
    void apply(double *out, const double *rhs) override;
    void apply_in_place(double *rhs) override;
};

struct CoarseCholOp : LinOp {
    DevBuf<double> inv;  // dense A^{-1}, row-major (n <= 8192)
    // above 8192 rows (chol.hip): the envelope Cholesky factor of the RCM-ordered
    // matrix in 64-row blocks -- off-diagonal slabs, inverses of the diagonal blocks
    int64_t nb = 0, env_bytes = 0;
    DevBuf<double> slab, mc, mr;
    DevBuf<int64_t> soff;
    DevBuf<int32_t> cmin, perm;
    mutable DevBuf<double> z;
    Kind kind() const override { return Kind::Coarse; }
    bool is_precond() const override { return true; }
    void apply(double *out, const double *rhs) override;
};

struct MgLevel {
    LinOpPtr A, S, R, P;  // R, P: transfer to the next-coarser level (null on the coarsest)
    // locality reordering (reorder.hip): the operators the caller added when A/S/R/P
    // above are renumbered copies; perm = the level's numbering (new -> original)
    LinOpPtr oA, oS, oR, oP;
    DevBuf<int32_t> perm;
    bool permuted = false;
    const LinOpPtr &origA() const { return oA ? oA : A; }
    const LinOpPtr &origS() const { return oS ? oS : S; }
    const LinOpPtr &origR() const { return oR ? oR : R; }
    const LinOpPtr &origP() const { return oP ? oP : P; }
    // device workspaces (allocated lazily at first apply)
    DevBuf<double> v, f, t, r;
};

struct MultigridOp : LinOp {
    std::vector<MgLevel> levels;
    int64_t mu = 1, steps = 1;
    bool use_graph = true;
    bool sgs_residual_form = false;  // true: literal smooth() order (residual SpMV + SGS(r))
    // s = 1 Jacobi levels: fold the first smoothing step from v = 0 (v = d*f)
    // into the residual (RESID0) and the correction (ADD0) instead of storing it
    bool fold_zero_guess = true;
    // R on wide grid-transfer classes writes the next level's first Jacobi step
    // from zero beside f_c (SPMV_SETDF) instead of a separate d*f pass
    bool restrict_df = true;
    // locality renumbering of general levels (reorder.hip): 0 off, 1 where it stays
    // bitwise and at least halves the x lines an SpMV slice touches (default), 2 every
    // eligible level
    int reorder = 1;
    std::mutex mtx;
    Kind kind() const override { return Kind::Multigrid; }
    bool is_precond() const override { return true; }
    void apply(double *out, const double *rhs) override;
    void add_level(LinOpPtr A, LinOpPtr S, LinOpPtr R, LinOpPtr P);
    void ensure_workspace();
    void invalidate_graphs();
    ~MultigridOp() override;

    // V-cycle building blocks (also used by the distributed multigrid)
    // pre_df: the restriction that produced f already wrote the first Jacobi
    // step from zero (d*f, SPMV_SETDF) into the level's t buffer
    void cycle(int64_t l, double *v, const double *f, bool v_zero, double *out_final, bool pre_df = false);
    void smooth(int64_t l, double *&v, double *&t, const double *f, bool v_zero, bool pre_df = false);
    // the renumbered fine level's rhs gather, with its first Jacobi step from zero
    // written beside it where the level takes that step unfolded
    void gather_fine(const double *rhs, hipStream_t s);
    // launch records of one V-cycle (eager, recorder on)
    std::vector<LaunchRec> cycle_plan();
    // one of the fine level's fused launches exactly as the cycle makes it, on the
    // cycle's workspace (which 0: folded residual + restriction into level 1's f
    // and t; 1: interpolation + post-smoothing from level 1's v into out); false
    // where the cycle does not take it (amg_multigrid_fine_launch: bench timing)
    bool fine_launch(int which, double *out, const double *rhs);
    // renumber eligible levels (first ensure_workspace) / restore the caller's operators
    void reorder_levels();
    void undo_reorder();
    // the same multigrid over the caller's operators (no renumbering)
    std::shared_ptr<MultigridOp> original_view();
    // the dense tail: with mu = 1 every level l >= tail_level is entered with v = 0,
    // so the part of the cycle from tail_level down (smoothing, residual,
    // restriction, the coarser levels, the coarsest solve, correction, post-
    // smoothing) maps that level's f to its v linearly: v = M f.  M (n x n,
    // row-major) is built once by running that part of the cycle on the n unit
    // vectors; the cycle then takes one GEMV there instead of its launches.
    // The first level 1 <= l < L - 1 with n_l <= flag dense_tail (0: off).
    int64_t tail_level = -1;
    void ensure_tail();
    // in-cycle timing of one fused fine-level launch (amg_multigrid_set_fine_timer)
    int fine_timer = -1;
    hipEvent_t fine_ev[2] = {nullptr, nullptr};

  private:
    struct GraphEntry {
        double *out;
        const double *rhs;
        hipGraphExec_t exec;
    };
    std::vector<GraphEntry> graphs_;
    uint64_t flags_gen_ = 0;  // flags_generation() the graphs were captured under
    bool workspace_ready_ = false;
    bool reorder_done_ = false;
    DevBuf<double> perm_f0_, perm_v0_;  // the fine level's rhs / result in its numbering
    DevBuf<double> tail_M_;
    uint64_t tail_key_ = ~uint64_t(0);
};
// out (n x n, row-major) = in^T
void dense_transpose(const double *in, double *out, int64_t n, hipStream_t s);
// v = e_j: zeros with a one at j
void unit_vector(double *v, int64_t n, int64_t j, hipStream_t s);
// y = x[p] / y[p] = x over n entries (reorder.hip; launch-plan records)
void perm_gather(double *out, const double *in, const int32_t *p, int64_t n, hipStream_t s);
void perm_scatter(double *out, const double *in, const int32_t *p, int64_t n, hipStream_t s);
// the gather and the first Jacobi step from zero in one pass: f0 = in[p], t = d * f0
void perm_gather_df(double *f0, double *t, const double *in, const int32_t *p, const DiagOp &D, int64_t n,
                    hipStream_t s);

// the zero-guess fold decision of one level (RESID0 + ADD0 instead of v = d*f)
// m's DIA codes are a constant 7- or 27-point stencil on an nx x ny x nz grid (nx
// even), truncated at the faces: fills m.dia_cst* (sgs27.hip)
bool dia_constant(GpuCsr &m);
bool fold_level(const CsrOp *A, const DiagOp *D, const CsrOp *P, bool fold_zero_guess, bool v_zero, int64_t steps);
// the restriction into a level writes that level's first Jacobi step from zero
// (SPMV_SETDF) -- false with FAMG_SETDF=0
bool setdf_enabled();
// R serves SPMV_SETDF (a grid-transfer overlay of either width, pattern SELL or 3x3 blocks)
inline bool r_has_setdf(const CsrOp *R) {
    return R && ((R->m.gtx_on && R->m.gtx_r) || (R->m.gtc_on && R->m.gtc_r) || R->m.kernel == SPMV_KERNEL_SELLP ||
                 R->m.kernel == SPMV_KERNEL_BSR);
}

// ---------------------------------------------------------------- factories

// sa_build_box(smoother = SGS): levels whose greedy coloring needs more colors
// than this get the L1 smoother instead (each color is one launch over 1/C of
// the rows: a dense Galerkin level with 20+ colors spent 1.6 ms of the 27-pt
// 256^3 V-cycle in latency-bound color launches, profiles/r02)
constexpr int64_t SGS_MAX_COLORS = 8;

CsrPtr make_csr(Ctx *ctx);
std::shared_ptr<DiagOp> make_jacobi(CsrOp &A, double omega);
std::shared_ptr<DiagOp> make_l1(CsrOp &A);
std::shared_ptr<DiagOp> make_l2(CsrOp &A);
std::shared_ptr<SgsOp> make_sgs(const CsrPtr &A, const int32_t *colors, bool validate = true);
// SGS over the owned rows of a distributed level (A: owned rows x [owned | ghost]
// columns; a row's columns keep the global order, so they need not ascend);
// colors: the global smoother's colors of those rows, ncolors the global count
// (every rank sweeps the same colors); aii: their diagonal (device, owned rows)
std::shared_ptr<SgsOp> make_sgs_slice(const CsrPtr &A, const int32_t *colors, int64_t ncolors, const double *aii);
// fused SGS phases for a 27-point grid operator stored as DIA codes (sgs27.hip)
// SgsOps built afterwards use the fused phases where they apply (default 1,
// FAMG_SGS_FUSED=0 sets 0; amg_set_sgs_fused)
extern int g_sgs_fused;
void sgs27_setup(SgsOp &S);
bool sgs27_applies(const SgsOp &S, const double *x, const double *b);  // fused and 16-B aligned vectors
void sgs27_sweep(SgsOp &S, double *x, const double *b, bool zero);
std::shared_ptr<CoarseCholOp> make_coarse_chol(CsrOp &A);

// SA setup pieces
CsrPtr sa_tentative(Ctx *ctx, int64_t n, const int64_t *agg_of, int64_t naggs,
                    const double *nn, double *coarse_nn);
CsrPtr smooth_interpolation(CsrOp &A, const CsrOp &P, double omega);
// Galerkin A_c = R (A P); grid: the coarse grid dims (hint for the x-staged
// stencil kernels) or null
CsrPtr galerkin_rap(const CsrOp &R, const CsrOp &A, const CsrOp &P, const int64_t *grid = nullptr);
CsrPtr transpose_op(const CsrOp &P);
CsrPtr spgemm_op(const CsrOp &A, const CsrOp &B);
void nn_stationary_l1(CsrOp &A, int64_t iters, double *x_host);
int64_t greedy_coloring(const GpuCsr &A, std::vector<int32_t> &color);
// BlockSmoother apply data: blocks in block-major row order, explicit inverses
// (column-major), chunks of <= 256 rows of whole blocks (block.hip).
struct BlockSmootherOp : LinOp {
    int64_t nblocks = 0, vdim = 1, max_block = 0, nchunks = 0;
    std::vector<int64_t> h_bptr;   // host copies (to_csr)
    std::vector<int32_t> h_rows;
    DevBuf<int32_t> rows;          // block-major original row ids (n)
    DevBuf<int32_t> blk_of;        // block of each block-major position (n)
    DevBuf<int64_t> bptr;          // nblocks+1
    DevBuf<int64_t> ioff;          // nblocks+1 offsets of the inverses
    DevBuf<int32_t> chunk;         // nchunks+1 position bounds (block aligned)
    DevBuf<double> inv;
    Kind kind() const override { return Kind::Block; }
    bool is_precond() const override { return true; }
    void apply(double *out, const double *rhs) override;
    void apply_in_place(double *rhs) override { apply(rhs, rhs); }
};
// BlockSmoother (block_smoothers.rs:80-291) over a node partition (ids 0..nagg-1,
// n/vdim nodes); blocks diagonally compensated and inverted exactly (block.hip).
std::shared_ptr<BlockSmootherOp> make_block_smoother(CsrOp &A, const int64_t *part, int64_t nagg, int64_t vdim);
std::shared_ptr<MultigridOp> sa_build_box(const CsrPtr &A, int64_t nx, int64_t ny, int64_t nz,
                                          int64_t bx, int64_t by, int64_t bz,
                                          int64_t coarsest_dim, int64_t max_levels,
                                          double omega, int smoother);

// ------------------------------------------------ general SA setup (sa.hip)

// Node-level strength graph (partitioners/mod.rs:337-393, block-reduced
// :294-301): CSR with strengths in (0, 1].
struct StrengthGraph {
    int64_t n = 0;
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    std::vector<double> w;
};
StrengthGraph strength_graph(const CsrOp &A, const double *nn, int64_t ld, int64_t k, const double *w,
                             int64_t depth, int64_t bs);
// MIS-seeded aggregates of a strength graph; returns the aggregate count
int64_t aggregate_mis(const StrengthGraph &G, std::vector<int64_t> &agg_of);
// tentative P for k candidates on nodes of bs dofs (interpolation/mod.rs:754-805)
CsrPtr sa_tentative_block(Ctx *ctx, int64_t nnodes, int64_t bs, const int64_t *agg_of, int64_t naggs,
                          const double *nn, int64_t ld, int64_t k, int64_t cd, double *coarse_nn);
// block_jacobi P smoothing (interpolation/mod.rs:963-1028)
CsrPtr block_jacobi_smooth(CsrOp &A, const CsrOp &P, int64_t bs, double omega);
// coarse near-null post-processing for k columns (hierarchy.rs:219-228)
void nn_postprocess(CsrOp &A, int64_t iters, double *x, int64_t ld, int64_t k);
struct SaConfig {
    int64_t block_size = 1, candidate_dimension = 1, strength_depth = 1, smoothing_steps = 1;
    int64_t coarsest_dim = 1000, max_levels = 0;
    double omega = 0.66;
    int smoother = 1;
};
struct SaLevelInfo {
    int64_t n, block_size, nodes, aggregates, strength_edges;
};
std::shared_ptr<MultigridOp> sa_build(const CsrPtr &A, const double *nn, int64_t ld, int64_t k,
                                      const double *weights, const SaConfig &cfg, std::vector<SaLevelInfo> *info);

}  // namespace famg
