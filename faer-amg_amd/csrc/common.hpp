// common.hpp -- runtime plumbing shared by the MI355X AMG library: status and
// error propagation, device buffers, the per-process device context.
//
// Errors are C++ exceptions inside the library (AmgError carrying an
// amg_status) and are converted to status codes + a thread-local message at the
// C ABI boundary (capi.cpp).  The reference panics instead.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/amg.h"

namespace famg {

struct AmgError : std::runtime_error {
    amg_status status;
    AmgError(amg_status s, const std::string &msg) : std::runtime_error(msg), status(s) {}
};

[[noreturn]] inline void fail(amg_status s, const std::string &msg) { throw AmgError(s, msg); }

#define FAMG_CHECK_HIP(expr)                                                               \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            ::famg::fail(e_ == hipErrorOutOfMemory ? AMG_ERR_OOM : AMG_ERR_HIP,            \
                         std::string(#expr) + ": " + hipGetErrorString(e_) + " at " +      \
                             __FILE__ + ":" + std::to_string(__LINE__));                   \
        }                                                                                  \
    } while (0)

#define FAMG_REQUIRE(cond, status, msg)                                                    \
    do {                                                                                   \
        if (!(cond)) ::famg::fail(status, msg);                                            \
    } while (0)

// Allocation policy: 0 (default) = hipMalloc.  1 = buffers of >= 16 MiB
// requested physically contiguous (hipDeviceMallocContiguous): measured
// UNSAFE on gfx950 -- with it, kernels on one stream read stale values written
// by the previous kernel (a SELL copy built from a half-updated smoothed P,
// 12 of 12 hierarchy builds, 0 of 12 with hipMalloc; scripts/dbg_p1d.py), so
// amg_set_alloc_policy(1) is refused.
extern int g_alloc_policy;

extern bool g_alloc_debug;  // FAMG_ALLOC_DEBUG=1: log large allocations to stderr

// FAMG_ALLOC_EXPERIMENT (root-causing the contiguous-allocation stale reads,
// DESIGN.md 3; never set in production): 1 = amg_set_alloc_policy(1) accepted,
// 2 = that plus a device-wide sync after each contiguous allocation
extern int g_alloc_experiment;
inline void *dev_alloc(size_t bytes) {
    void *p = nullptr;
    const bool large = bytes >= (size_t(16) << 20);
    if (g_alloc_policy == 1 && large) {
        if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) == hipSuccess && p) {
            if (g_alloc_debug) fprintf(stderr, "famg alloc contiguous %p %zu\n", p, bytes);
            // root-cause experiment (scripts/alloc_coherence.py): 2 = device-wide
            // sync right after the allocation, before any kernel touches it
            if (g_alloc_experiment == 2) FAMG_CHECK_HIP(hipDeviceSynchronize());
            return p;
        }
        (void)hipGetLastError();
        p = nullptr;
    }
    FAMG_CHECK_HIP(hipMalloc(&p, bytes));
    if (g_alloc_debug && large) fprintf(stderr, "famg alloc plain %p %zu\n", p, bytes);
    return p;
}

// Owning device allocation.  Sizes are in elements.  Allocation and free are
// synchronous (setup-time only; nothing in an apply path allocates).
template <typename T> class DevBuf {
  public:
    DevBuf() = default;
    explicit DevBuf(size_t n) { resize(n); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    // pad: extra elements allocated past n (vector loads may read up to 16 B past the end)
    void resize(size_t n, size_t pad = 0) {
        release();
        if (n + pad) p_ = static_cast<T *>(dev_alloc((n + pad) * sizeof(T)));
        n_ = n;
    }
    void release() {
        if (p_) (void)hipFree(p_);
        p_ = nullptr;
        n_ = 0;
    }
    T *get() const { return p_; }
    size_t size() const { return n_; }
    size_t bytes() const { return n_ * sizeof(T); }

  private:
    T *p_ = nullptr;
    size_t n_ = 0;
};

// One per process / device (one process per GPU).  All work of the handles
// created under a context is ordered on `stream`.
struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 256;
    // scratch used by host-memory staging and reductions
    DevBuf<double> red_partials;   // block partial sums for deterministic reductions
    DevBuf<double> red_result;     // reduction results
    double *host_red = nullptr;    // pinned host mirror of red_result
    void set_device() const { FAMG_CHECK_HIP(hipSetDevice(device)); }
    ~Ctx();
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Run-time A/B switches that change which kernels a cycle launches (bitwise
// neutral).  Read once from the environment (FAMG_FOLD_XSCS, FAMG_DIA_DK,
// FAMG_VEC_WPR) into these flags; amg_set_flag changes one and bumps
// g_flags_gen, which makes every multigrid drop the hipGraphs it captured under
// the old value (a graph replays the launches it recorded).
enum FlagId : int { FLAG_FOLD_XSCS = 0, FLAG_DIA_DK = 1, FLAG_VEC_WPR = 2, FLAG_GTX_TIME = 3, FLAG_SGS27_MARCH = 4, FLAG_XS_PIPE = 5,
              FLAG_BSR_KERNEL = 6, FLAG_BSR_LONG = 7,
              FLAG_DIA7_RP = 8, FLAG_FINE_FUSE = 9, FLAG_DENSE_TAIL = 10, FLAG_COUNT = 11 };
int64_t flag(FlagId f);
void set_flag(FlagId f, int64_t v);
uint64_t flags_generation();

// Launch plan (amg_multigrid_cycle_plan): while g_launch_log is set on this
// thread, every kernel the V-cycle launches appends one record with the
// algorithmic bytes of that launch (the bytes its storage streams
// + the vectors it reads and writes) and its 32-bit-CSR equivalent.  The
// records come from the code that issues the launches, so fold decisions,
// SGS colour launches and storage choices are what actually ran.
struct LaunchRec {
    int32_t level, role, kernel, mode;
    int64_t rows, bytes, csr_bytes;
    const char *name;
};
struct LaunchLog {
    std::vector<LaunchRec> recs;
    int32_t level = 0, role = AMG_ROLE_OTHER;
    int32_t level_base = 0;  // added to log_at's level (a distributed cycle's redundant tail)
};
extern thread_local LaunchLog *g_launch_log;
inline void log_launch(const char *name, int32_t kernel, int32_t mode, int64_t rows, int64_t bytes,
                       int64_t csr_bytes = -1) {
    if (g_launch_log)
        g_launch_log->recs.push_back({g_launch_log->level, g_launch_log->role, kernel, mode, rows, bytes,
                                      csr_bytes < 0 ? bytes : csr_bytes, name});
}
inline void log_at(int64_t level, int32_t role) {
    if (g_launch_log) {
        g_launch_log->level = g_launch_log->level_base + (int32_t)level;
        g_launch_log->role = role;
    }
}

}  // namespace famg
