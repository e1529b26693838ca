"""Rank body of tests/test_gpu_rccl_multi.py (launched by torch.distributed.run,
one rank per GPU, RCCL communicator): a 7-point 64 x 64 x (32 N) box hierarchy on
z-slabs, the distributed cycle eager and as a replayed hipGraph with the
halo/interior overlap on and off, compared bitwise on every rank, and a second
(out, rhs) pair replayed through its own graph.  Prints one JSON line per rank."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(local, stream=stream.cuda_stream)
    dims = (64, 64, 32 * world)
    A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    splits = fa.slab_splits(fa.box_level_dims(dims, (2, 2, 2), mg.levels()), world)
    obj = [fa.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = fa.Comm(ctx, nranks=world, rank=rank, uid=obj[0])
    dm = fa.DistMultigrid(comm, mg, splits, agglomerate_rows=1000)
    r0, r1 = dm.local_rows()
    rng = np.random.default_rng(5)
    b1 = torch.as_tensor(rng.uniform(-1, 1, A.nrows)[r0:r1].copy(), device=f"cuda:{local}")
    b2 = torch.as_tensor(rng.uniform(-1, 1, A.nrows)[r0:r1].copy(), device=f"cuda:{local}")
    res = {"rank": rank, "world": world}
    ok = True
    for overlap in (True, False):
        dm.set_overlap(overlap)
        dm.set_graph(False)
        e1, e2 = torch.empty_like(b1), torch.empty_like(b2)
        dm.apply(e1, b1)
        dm.apply(e2, b2)
        dm.set_graph(True)
        g1, g2 = torch.empty_like(b1), torch.empty_like(b2)
        for _ in range(2):  # capture + replay, per (out, rhs) pair
            dm.apply(g1, b1)
            dm.apply(g2, b2)
        torch.cuda.synchronize()
        same = bool(torch.equal(e1, g1) and torch.equal(e2, g2))
        res[f"overlap_{overlap}"] = same
        ok = ok and same
    dm.set_graph(False)
    # overlap is bitwise neutral too
    dm.set_overlap(True)
    z_on = torch.empty_like(b1)
    dm.apply(z_on, b1)
    dm.set_overlap(False)
    z_off = torch.empty_like(b1)
    dm.apply(z_off, b1)
    torch.cuda.synchronize()
    res["overlap_neutral"] = bool(torch.equal(z_on, z_off))
    ok = ok and res["overlap_neutral"]
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    res["all_ranks_ok"] = float(t[0]) == 1.0
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
