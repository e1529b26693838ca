// handles.hpp -- definitions of the opaque C-ABI handle types and the shared
// error plumbing of the extern "C" layer (capi.cpp, dist.hip).
#pragma once

#include "famg.hpp"

struct amg_ctx {
    famg::Ctx ctx;  // must stay the first member (Ctx* <-> amg_ctx* casts)
    famg::DevBuf<double> stage_in, stage_out;  // host-memory staging
    hipEvent_t join_event = nullptr;            // amg_ctx_join_stream
    ~amg_ctx() {
        if (join_event) (void)hipEventDestroy(join_event);
    }
};

struct amg_linop {
    famg::LinOpPtr op;
};

// host CSR (loaders, generators, strength graphs): int64 indices, fp64 values
struct amg_host_csr {
    int64_t nrows = 0, ncols = 0;
    std::vector<int64_t> rp, ci;
    std::vector<double> va;
};

namespace famg {
// record the thread-local message returned by amg_last_error(); returns s
amg_status set_last_error(amg_status s, const char *msg);

// copy launch records into the caller's amg_launch_rec array (cycle plans)
void export_plan(const std::vector<LaunchRec> &plan, amg_launch_rec *recs, int64_t cap, int64_t *count);

template <typename F> amg_status guard(F &&f) {
    try {
        f();
        set_last_error(AMG_OK, "");
        return AMG_OK;
    } catch (const AmgError &e) {
        return set_last_error(e.status, e.what());
    } catch (const std::bad_alloc &) {
        return set_last_error(AMG_ERR_OOM, "host allocation failed");
    } catch (const std::exception &e) {
        return set_last_error(AMG_ERR_INVALID, e.what());
    }
}
}  // namespace famg
