// blas1.hip -- vector kernels of the V-cycle and solve drivers.
//
// The reference's dense vector work (`f - work`, `v += work`, Diag scaling,
// faer CG dots/axpys; multigrid.rs:266,342,350,420-422; utils.rs:600-626) runs
// here on HBM-resident vectors.  Streaming element-wise kernels use 16-byte
// (2 x fp64) accesses per lane; reductions are deterministic (fixed grid, fixed
// tree) so repeated solves are bitwise reproducible.
#include "famg.hpp"

namespace famg {

typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int EW_BS = 256;

static inline unsigned ew_grid(int64_t n2) {
    int64_t g = ceil_div(n2, EW_BS);
    if (g > 65536) g = 65536;
    return static_cast<unsigned>(g < 1 ? 1 : g);
}

// Element-wise kernels: Op(i) over [0,n); vectorized by 2 with a scalar tail.
#define FAMG_EW_KERNEL(NAME, PARAMS, BODY)                                                 \
    __global__ __launch_bounds__(EW_BS) void NAME PARAMS {                                 \
        const int64_t stride = (int64_t)gridDim.x * EW_BS;                                 \
        for (int64_t i = (int64_t)blockIdx.x * EW_BS + threadIdx.x; i < n; i += stride) {  \
            BODY;                                                                          \
        }                                                                                  \
    }

FAMG_EW_KERNEL(k_fill, (double *x, double v, int64_t n), x[i] = v)
FAMG_EW_KERNEL(k_copy, (double *dst, const double *src, int64_t n), dst[i] = src[i])
FAMG_EW_KERNEL(k_sub, (double *o, const double *a, const double *b, int64_t n), o[i] = a[i] - b[i])
FAMG_EW_KERNEL(k_add, (double *x, const double *y, int64_t n), x[i] = x[i] + y[i])
FAMG_EW_KERNEL(k_mul, (double *o, const double *d, const double *a, int64_t n), o[i] = d[i] * a[i])
FAMG_EW_KERNEL(k_axpy, (double *y, double al, const double *x, int64_t n), y[i] = y[i] + al * x[i])
FAMG_EW_KERNEL(k_xpay, (double *y, double be, const double *x, int64_t n), y[i] = x[i] + be * y[i])
FAMG_EW_KERNEL(k_scale, (double *x, double al, int64_t n), x[i] = x[i] * al)
FAMG_EW_KERNEL(k_nn_step, (double *x, const double *d, const double *r, int64_t n),
               { const double o = d[i] * (x[i] - r[i]); x[i] = x[i] + o; })

// 2-wide versions of the hottest element-wise ops (x*d, a-b) for the V-cycle
__global__ __launch_bounds__(EW_BS) void k_mul2(dbl2 *o, const dbl2 *d, const dbl2 *a, int64_t n2) {
    const int64_t stride = (int64_t)gridDim.x * EW_BS;
    for (int64_t i = (int64_t)blockIdx.x * EW_BS + threadIdx.x; i < n2; i += stride) o[i] = d[i] * a[i];
}

// out = dt[dc] * a, two elements per lane (16-B accesses of out and a)
__global__ __launch_bounds__(EW_BS) void k_mul2_coded(dbl2 *o, const uint8_t *dc, const double *dt, const dbl2 *a,
                                                      int64_t n2) {
    const int64_t stride = (int64_t)gridDim.x * EW_BS;
    for (int64_t i = (int64_t)blockIdx.x * EW_BS + threadIdx.x; i < n2; i += stride) {
        const dbl2 d = {dt[dc[2 * i]], dt[dc[2 * i + 1]]};
        o[i] = d * a[i];
    }
}
FAMG_EW_KERNEL(k_mul_coded, (double *o, const uint8_t *dc, const double *dt, const double *a, int64_t n),
               o[i] = dt[dc[i]] * a[i])

void vec_mul_coded(double *o, const uint8_t *dc, const double *dt, const double *a, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    log_launch("vec_mul_coded", -1, -1, n, 17 * n);
    const bool aligned = ((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(a)) & 15) == 0;
    if (aligned && n >= 2) {
        const int64_t n2 = n / 2;
        hipLaunchKernelGGL(k_mul2_coded, dim3(ew_grid(n2)), dim3(EW_BS), 0, s, (dbl2 *)o, dc, dt, (const dbl2 *)a, n2);
        if (n & 1)
            hipLaunchKernelGGL(k_mul_coded, dim3(1), dim3(EW_BS), 0, s, o + n - 1, dc + n - 1, dt, a + n - 1, (int64_t)1);
    } else {
        hipLaunchKernelGGL(k_mul_coded, dim3(ew_grid(n)), dim3(EW_BS), 0, s, o, dc, dt, a, n);
    }
}

void vec_fill(double *x, double v, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_fill", -1, -1, n, 8 * n);
    if (n > 0) hipLaunchKernelGGL(k_fill, dim3(ew_grid(n)), dim3(EW_BS), 0, s, x, v, n);
}
void vec_copy(double *dst, const double *src, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_copy", -1, -1, n, 16 * n);
    if (n > 0) FAMG_CHECK_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, s));
}
void vec_sub(double *o, const double *a, const double *b, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_sub", -1, -1, n, 24 * n);
    if (n > 0) hipLaunchKernelGGL(k_sub, dim3(ew_grid(n)), dim3(EW_BS), 0, s, o, a, b, n);
}
void vec_add_inplace(double *x, const double *y, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_add", -1, -1, n, 24 * n);
    if (n > 0) hipLaunchKernelGGL(k_add, dim3(ew_grid(n)), dim3(EW_BS), 0, s, x, y, n);
}
void vec_mul(double *o, const double *d, const double *a, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    log_launch("vec_mul", -1, -1, n, 24 * n);
    const bool aligned = ((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(d) |
                           reinterpret_cast<uintptr_t>(a)) & 15) == 0;
    if (aligned && n >= 2) {
        const int64_t n2 = n / 2;
        hipLaunchKernelGGL(k_mul2, dim3(ew_grid(n2)), dim3(EW_BS), 0, s, (dbl2 *)o,
                           (const dbl2 *)d, (const dbl2 *)a, n2);
        if (n & 1) hipLaunchKernelGGL(k_mul, dim3(1), dim3(EW_BS), 0, s, o + n - 1, d + n - 1, a + n - 1, (int64_t)1);
    } else {
        hipLaunchKernelGGL(k_mul, dim3(ew_grid(n)), dim3(EW_BS), 0, s, o, d, a, n);
    }
}
void vec_axpy(double *y, double al, const double *x, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_axpy", -1, -1, n, 24 * n);
    if (n > 0) hipLaunchKernelGGL(k_axpy, dim3(ew_grid(n)), dim3(EW_BS), 0, s, y, al, x, n);
}
void vec_xpay(double *y, double be, const double *x, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_xpay", -1, -1, n, 24 * n);
    if (n > 0) hipLaunchKernelGGL(k_xpay, dim3(ew_grid(n)), dim3(EW_BS), 0, s, y, be, x, n);
}
void vec_scale(double *x, double al, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_scale", -1, -1, n, 16 * n);
    if (n > 0) hipLaunchKernelGGL(k_scale, dim3(ew_grid(n)), dim3(EW_BS), 0, s, x, al, n);
}
void vec_nn_step(double *x, const double *d, const double *r, int64_t n, hipStream_t s) {
    if (n > 0) log_launch("vec_nn_step", -1, -1, n, 32 * n);
    if (n > 0) hipLaunchKernelGGL(k_nn_step, dim3(ew_grid(n)), dim3(EW_BS), 0, s, x, d, r, n);
}

// ---------------------------------------------------------------- reductions

constexpr int RED_GRID = VEC_DOT_PARTIALS;

__device__ __forceinline__ double block_sum(double v, double *sh) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < (int)(blockDim.x >> 6); k++) t += sh[k];
    return t;
}

__global__ __launch_bounds__(256) void k_dot_partial(const double *x, const double *y, int64_t n,
                                                     double *partials) {
    __shared__ double sh[4];
    double acc = 0.0;
    const int64_t stride = (int64_t)RED_GRID * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        acc = fma(x[i], y[i], acc);
    const double t = block_sum(acc, sh);
    if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_dot_final(const double *partials, double *res) {
    __shared__ double sh[4];
    double acc = 0.0;
    for (int i = threadIdx.x; i < RED_GRID; i += 256) acc += partials[i];
    const double t = block_sum(acc, sh);
    if (threadIdx.x == 0) *res = t;
}

void vec_dot_dev(const double *x, const double *y, int64_t n, double *res, double *partials, hipStream_t s) {
    log_launch("vec_dot", -1, -1, n, 16 * n);
    hipLaunchKernelGGL(k_dot_partial, dim3(RED_GRID), dim3(256), 0, s, x, y, n, partials);
    hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(256), 0, s, partials, res);
    FAMG_CHECK_HIP(hipGetLastError());
}

void vec_dot_dev(const double *x, const double *y, int64_t n, double *res, Ctx &ctx) {
    if (ctx.red_partials.size() < (size_t)RED_GRID) ctx.red_partials.resize(RED_GRID);
    vec_dot_dev(x, y, n, res, ctx.red_partials.get(), ctx.stream);
}

double vec_dot(const double *x, const double *y, int64_t n, Ctx &ctx) {
    if (ctx.red_result.size() < 8) ctx.red_result.resize(8);
    if (!ctx.host_red) FAMG_CHECK_HIP(hipHostMalloc((void **)&ctx.host_red, 8 * sizeof(double)));
    vec_dot_dev(x, y, n, ctx.red_result.get(), ctx);
    FAMG_CHECK_HIP(hipMemcpyAsync(ctx.host_red, ctx.red_result.get(), sizeof(double),
                                  hipMemcpyDeviceToHost, ctx.stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(ctx.stream));
    return ctx.host_red[0];
}

// ------------------------------------------------------------- dense GEMV

// out = M x, M row-major n x n: one wave per row, 2 x fp64 per lane.
__global__ __launch_bounds__(256) void k_gemv(const double *M, const double *x, double *out, int64_t n) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const double *mr = M + row * n;
    double acc = 0.0;
    for (int64_t j = lane; j < n; j += 64) acc = fma(mr[j], x[j], acc);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) out[row] = acc;
}

// The same for even n: 16-B loads of M and x, eight of them in flight per lane
// before the first fma (the dense tail's 4096 x 4096 M streams 134 MB per cycle)
typedef double gemv_dbl2_t __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_gemv2(const double *M, const double *x, double *out, int64_t n) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const double *mr = M + row * n;
    double a0 = 0.0, a1 = 0.0;
    constexpr int U = 8;
    for (int64_t j0 = 2 * lane; j0 < n; j0 += 128 * U) {
        gemv_dbl2_t m[U], xx[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t j = min(j0 + 128 * u, n - 2);
            m[u] = __builtin_nontemporal_load(reinterpret_cast<const gemv_dbl2_t *>(mr + j));
            xx[u] = *reinterpret_cast<const gemv_dbl2_t *>(x + j);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (j0 + 128 * u < n) {
                a0 = fma(m[u].x, xx[u].x, a0);
                a1 = fma(m[u].y, xx[u].y, a1);
            }
    }
    double acc = a0 + a1;
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) out[row] = acc;
}

void dense_gemv(const double *M, const double *x, double *out, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    log_launch("gemv", -1, -1, n, 8 * n * n + 16 * n);
    if (n % 2 == 0 && n >= 2) hipLaunchKernelGGL(k_gemv2, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s, M, x, out, n);
    else hipLaunchKernelGGL(k_gemv, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s, M, x, out, n);
    FAMG_CHECK_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_transpose(const double *in, double *out, int64_t n) {
    __shared__ double t[32][33];
    const int64_t bx = (int64_t)blockIdx.x * 32, by = (int64_t)blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int k = ty; k < 32; k += 8)
        if (by + k < n && bx + tx < n) t[k][tx] = in[(by + k) * n + bx + tx];
    __syncthreads();
    for (int k = ty; k < 32; k += 8)
        if (bx + k < n && by + tx < n) out[(bx + k) * n + by + tx] = t[tx][k];
}

void dense_transpose(const double *in, double *out, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    const dim3 grid((unsigned)ceil_div(n, 32), (unsigned)ceil_div(n, 32));
    hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, s, in, out, n);
    FAMG_CHECK_HIP(hipGetLastError());
}

__global__ void k_unit(double *v, int64_t n, int64_t j) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i == j ? 1.0 : 0.0;
}

void unit_vector(double *v, int64_t n, int64_t j, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_unit, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, v, n, j);
    FAMG_CHECK_HIP(hipGetLastError());
}

// ------------------------------------------------------------------- scan

constexpr int SCAN_BS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_CHUNK = SCAN_BS * SCAN_ITEMS;

__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t *sh, int64_t *total) {
    // inclusive scan within the wave
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int64_t wpre = 0, tot = 0;
    for (int k = 0; k < SCAN_BS / 64; k++) {
        if (k < w) wpre += sh[k];
        tot += sh[k];
    }
    __syncthreads();
    *total = tot;
    return wpre + x - v;
}

__global__ __launch_bounds__(SCAN_BS) void k_scan_sums(const int64_t *in, int64_t n, int64_t *sums) {
    __shared__ int64_t sh[SCAN_BS / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK + threadIdx.x * SCAN_ITEMS;
    int64_t s = 0;
    for (int k = 0; k < SCAN_ITEMS; k++)
        if (base + k < n) s += in[base + k];
    int64_t tot;
    block_exclusive_scan(s, sh, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// single block: exclusive scan of nb block sums in place; writes grand total
__global__ __launch_bounds__(SCAN_BS) void k_scan_top(int64_t *sums, int64_t nb, int64_t *total_out) {
    __shared__ int64_t sh[SCAN_BS / 64];
    int64_t carry = 0;
    for (int64_t base = 0; base < nb; base += SCAN_BS) {
        const int64_t i = base + threadIdx.x;
        const int64_t v = i < nb ? sums[i] : 0;
        int64_t tot;
        const int64_t ex = block_exclusive_scan(v, sh, &tot);
        if (i < nb) sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total_out = carry;
}

__global__ __launch_bounds__(SCAN_BS) void k_scan_apply(const int64_t *in, int64_t n,
                                                        const int64_t *sums, int64_t *out) {
    __shared__ int64_t sh[SCAN_BS / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK + threadIdx.x * SCAN_ITEMS;
    int64_t vals[SCAN_ITEMS];
    int64_t s = 0;
    for (int k = 0; k < SCAN_ITEMS; k++) {
        vals[k] = base + k < n ? in[base + k] : 0;
        s += vals[k];
    }
    int64_t tot;
    int64_t ex = block_exclusive_scan(s, sh, &tot) + sums[blockIdx.x];
    for (int k = 0; k < SCAN_ITEMS; k++) {
        if (base + k < n) out[base + k] = ex;
        ex += vals[k];
    }
}

int64_t scan_counts(const int64_t *counts, int64_t *out, int64_t n, Ctx &ctx) {
    const int64_t nb = ceil_div(n, SCAN_CHUNK);
    DevBuf<int64_t> sums(nb + 1);
    hipStream_t s = ctx.stream;
    if (n > 0) {
        hipLaunchKernelGGL(k_scan_sums, dim3((unsigned)nb), dim3(SCAN_BS), 0, s, counts, n, sums.get());
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_BS), 0, s, sums.get(), nb, out + n);
        hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(SCAN_BS), 0, s, counts, n, sums.get(), out);
        FAMG_CHECK_HIP(hipGetLastError());
    } else {
        FAMG_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), s));
    }
    int64_t total = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&total, out + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return total;
}

}  // namespace famg
