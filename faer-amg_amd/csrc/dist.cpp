// dist.cpp -- multi-GPU row-block partition + RCCL halo exchange (placeholder:
// filled in by the distributed milestone).
#include "famg.hpp"

using namespace famg;

extern "C" {
int32_t amg_comm_unique_id_size(void) { return 128; }
amg_status amg_comm_get_unique_id(void *) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_comm_create(amg_ctx *, int32_t, int32_t, const void *, amg_comm **) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_comm_destroy(amg_comm *) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_comm_barrier(amg_comm *) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_comm_allreduce_max(amg_comm *, double *) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_dist_csr_create(amg_comm *, const amg_linop *, const int64_t *, const int64_t *, amg_linop **) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_dist_plan_info(const amg_linop *, int64_t *) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_dist_multigrid_create(amg_comm *, const amg_linop *, int64_t, amg_linop **) { return AMG_ERR_UNSUPPORTED; }
amg_status amg_dist_local_rows(const amg_linop *, int64_t *, int64_t *) { return AMG_ERR_UNSUPPORTED; }
}
