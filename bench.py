"""Benchmark: AMG V-cycle apply on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Step = one V-cycle (Multigrid::apply, reference multigrid.rs:469) of the
smoothed-aggregation hierarchy of the 3-D 7-point Laplacian (config C2:
2^3 box aggregates, one constant candidate, weighted Jacobi omega = 0.66,
s = 1, mu = 1, Cholesky coarsest), b ~ U(-1,1) from splitmix64 seed 42,
x0 = 0.  Matrices and vectors are generated on the device and resident in
HBM before timing.

N = 1: the 256^3 problem on one GPU.
N > 1: weak scaling -- the global grid has N x 256^3 rows (N = 2: 256x256x512,
4: 256x512x512, 8: 512^3 = config C4), every level is cut into N z-slabs
(one per rank, RCCL halo exchange over xGMI before each SpMV), levels below
--agglomerate rows are gathered and cycled redundantly on every rank.
value = global V-cycles/s x N  (= 256^3-equivalent V-cycles/s, whole job).

Prints ONE JSON line on rank 0 (stdout); diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "V-cycles/s + fine-level SpMV GB/s vs HBM peak, 3D 7-pt Laplacian 256³"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def splitmix_uniform(n, seed=42):
    """b ~ U(-1,1): z_i = splitmix64(seed + (i+1)*golden), u = (z>>11)*2^-53, b = 2u-1."""
    import numpy as np
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def csr_traffic():
    """HBM bytes per launch of roofline.csr's SpMV from the latest committed PMC
    passes (scripts/pmc_csr.sh -> profiles/rNN/csr_spmv_traffic.json), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "csr_spmv_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def measured_traffic(edge, problem):
    """HBM bytes per fine-SpMV launch from the committed rocprofv3 PMC passes
    (scripts/pmc_fine_spmv.py + scripts/pmc_summary.py; FETCH_SIZE calibrated on
    a diagonal matrix through the same kernel).  None if not measured for this
    workload."""
    import glob
    if problem == "elast" and edge == 80:  # the C5 stand-in's renumbered fine SpMV (scripts/pmc_bsr_renum.sh)
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "c5_renum_spmv_traffic.json")))
        if not files:
            return None, None
        d = json.load(open(files[-1]))
        return d["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    if edge != 256 or problem != "7pt":
        return None, None
    # the latest round's cycle-wide passes (scripts/pmc_cycle.sh: the roofline
    # kernel -- DIA SET on A_0 -- and every launch of the cycle), else the
    # older fine-SpMV-only passes
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "c2_cycle_traffic.json")))
    if files:
        d = json.load(open(files[-1]))
        return d["fine_set"]["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "fine_spmv_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def spmv_bytes(nrows, ncols, nnz):
    """Algorithmic bytes of y = A x in CSR with 32-bit indices."""
    return 12 * nnz + 4 * (nrows + 1) + 8 * ncols + 8 * nrows


def spmv_bytes_fmt(M):
    """Algorithmic bytes of y = M x in the storage the library chose for M: the
    matrix bytes that format streams (SELL-64 values + compressed column indices
    + slice metadata, or CSR) + x read once + y written."""
    m, n = M.dims()
    return M.spmv_info()["stream_bytes"] + 8 * n + 8 * m


def time_kernel(fn, iters, stream):
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


def weak_dims(n, N):
    """N x n^3 rows: double z, then y, then x for powers of two; z-stack otherwise."""
    d = [n, n, n]
    if N & (N - 1) == 0:
        k, ax = N, 2
        while k > 1:
            d[ax] *= 2
            ax = (ax - 1) % 3
            k //= 2
    else:
        d[2] *= N
    return tuple(d)


def oracle_levels(mg, smoother):
    """The GPU hierarchy's arrays (A_l, R_l, P_l exactly as the V-cycle uses them)
    as oracle levels, with the smoother each level actually got."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    levels = []
    nl = mg.levels()
    for l in range(nl):
        Al, Sl, Rl, Pl = mg.level(l)
        kind = Sl.kind
        d = {"A": O.Csr.from_arrays(*Al.dims(), *Al.arrays())}
        if l == nl - 1:
            d["smoother"] = "chol"
        elif kind == "sgs":
            d["smoother"] = "sgs"
        elif kind == "diag":
            d["smoother"] = "jacobi" if smoother == "jacobi" else "l1"
        elif kind == "block":
            # BlockSmoother::into_sparse_mat (block_smoothers.rs:122-146)
            M = fa_block_to_csr(Sl)
            d["smoother"] = ("csr", O.Csr.from_arrays(*M.dims(), *M.arrays()))
        else:
            raise ValueError(f"no CPU restatement of the {kind} smoother")
        if Rl is not None:
            d["R"] = O.Csr.from_arrays(*Rl.dims(), *Rl.arrays())
            d["P"] = O.Csr.from_arrays(*Pl.dims(), *Pl.arrays())
        levels.append(d)
    return levels


def fa_block_to_csr(S):
    import faer_amg_amd as fa
    h = fa.vp()
    fa._ck(fa.lib().amg_block_smoother_to_csr(S.h, fa.C.byref(h)))
    return fa.SparseMatOp(h, S.ctx)


def cgroup_cpu_quota():
    """CPUs this process's cgroup may use (cpu.max quota / period), None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def _time_cycles(omg, b, budget_s, max_cycles=60, min_cycles=3):
    """Per-V-cycle wall times of the oracle (after one warm-up cycle)."""
    import numpy as np
    import oracle as O
    out = np.empty_like(b)
    O.lib().orc_mg_apply(omg.h, b, out)  # warm-up (page faults, ParSpmm tiles)
    ts = []
    t_end = time.perf_counter() + budget_s
    while len(ts) < max_cycles and (len(ts) < min_cycles or time.perf_counter() < t_end):
        t0 = time.perf_counter()
        O.lib().orc_mg_apply(omg.h, b, out)
        ts.append(time.perf_counter() - t0)
    return ts, out


def cpu_side(mg, A, b_host, z_gpu, args, hist_gpu=None, rho_cycles=10, min_cycles=None, budget=None,
             what_gpu="GPU"):
    """Everything the CPU restatement contributes to the bench line, on the SAME
    hierarchy (the GPU's A_l, R_l, P_l arrays):
      parity      -- ||z_gpu - z_oracle|| / ||z_oracle|| for one V-cycle (<= 1e-11,
                     SURVEY.md 8(c)) and rho_k of 10 stationary cycles GPU vs oracle
      cpu_baseline -- the reference's rayon path restated (ParSpmmOp 8192x8192 CSC
                     tiles with usize indices, per-call temporaries; par_spmm.rs,
                     multigrid.rs:251-424): median V-cycle time at 16 threads
                     (Par::Rayon(16), examples/amg/main.rs:227) and at all host cores,
                     plus the fine-level ParSpmm SpMV in GB/s."""
    import numpy as np
    import torch
    import faer_amg_amd as fa
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    t_imp = time.perf_counter()
    levels = oracle_levels(mg, args.smoother)
    omg = O.Multigrid(levels)
    OA = levels[0]["A"]
    log(f"oracle hierarchy import {time.perf_counter() - t_imp:.1f}s")
    nproc = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    # every host core this process may run on: nproc capped by the cgroup CPU
    # quota (256 threads inside a 16-CPU quota measured oversubscription)
    all_threads = max(1, min(nproc, int(quota))) if quota else nproc
    t16 = args.cpu_threads

    # parity of one V-cycle (the bench's own z from the timed loop); >= 50 cycles
    # at 16 threads (median over >= 50 cycles)
    omg.set_parallel(t16)
    ts16, zref = _time_cycles(omg, b_host, args.cpu_budget if budget is None else budget,
                              min_cycles=args.cpu_min_cycles if min_cycles is None else min_cycles)
    rel_err = float(np.linalg.norm(z_gpu - zref) / np.linalg.norm(zref))
    # residual history of K stationary cycles (simple_geometric.rs:117-158)
    K = rho_cycles
    if hist_gpu is None:
        bd = torch.as_tensor(b_host, device=torch.cuda.current_device())
        xd = torch.zeros_like(bd)
        _, hist_gpu = fa.stationary_solve(A, mg, bd, xd, max_iter=K + 1, rel_tol=1e-300)
        torch.cuda.synchronize()
    hist_gpu = np.asarray(hist_gpu, np.float64)[:K + 1]
    _, _, hist_cpu = O.stationary_solve(OA, omg, b_host, max_iter=K + 1, rel_tol=1e-300)
    rho_rel = float(np.max(np.abs(hist_gpu - hist_cpu) / hist_cpu))

    # fine-level SpMV of the restated rayon path (ParSpmmOp), 16 threads
    par = O.ParSpmm(OA)
    x = np.ones(OA.ncols)
    par.apply(x)
    tsp = []
    for _ in range(5):
        t0 = time.perf_counter()
        par.apply(x)
        tsp.append(time.perf_counter() - t0)
    m, n, nnz = OA.dims()
    spmv_t = float(np.median(tsp))
    del par

    res = {"value": round(1.0 / float(np.median(ts16)), 4), "unit": "V-cycles/s", "cores": t16,
           "kind": "port",
           "sample": f"median of {len(ts16)} V-cycles of the same hierarchy as the GPU run "
                     f"(oracle restatement of the rayon path: ParSpmmOp 8192x8192 CSC tiles, "
                     f"usize indices, per-call temporaries; OpenMP {t16} threads = Par::Rayon(16))",
           "fine_spmv_ms": round(spmv_t * 1e3, 3),
           "fine_spmv_GBs_32bit_formula": round(spmv_bytes(m, n, nnz) / spmv_t / 1e9, 2),
           "fine_spmv_GBs_usize_layout": round((16 * nnz + 8 * (m + 1) + 8 * n + 8 * m) / spmv_t / 1e9, 2)}
    if all_threads != t16:
        omg.set_parallel(all_threads)
        tsa, _ = _time_cycles(omg, b_host, args.cpu_budget / 2, min_cycles=3)
        res["all_cores"] = {"value": round(1.0 / float(np.median(tsa)), 4), "cores": all_threads,
                            "nproc": nproc, "cpu_quota": quota,
                            "sample": f"median of {len(tsa)} V-cycles at {all_threads} OpenMP threads"}
        omg.set_parallel(t16)
    parity = {"vcycle_rel_err": rel_err, "tol": 1e-11, "ok": rel_err <= 1e-11 and rho_rel <= 1e-8,
              "rho_k_gpu": [float(v) for v in hist_gpu], "rho_k_cpu": [float(v) for v in hist_cpu],
              "rho_k_max_rel_diff": rho_rel, "rho_k_tol": 1e-8, "rho_k_cycles": K,
              "what": f"one V-cycle z = M b and {K} stationary cycles (rho_k = ||b - A x_k||/||b||), "
                      f"{what_gpu} vs the oracle restatement on the same hierarchy"}
    return res, parity


def make_operator(fa, ctx, args, dims):
    """The fine operator of the workload (device-resident)."""
    if args.problem == "7pt":
        return fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
    if args.problem == "27pt":
        return fa.SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    if args.problem == "elast":  # in-tree C5 stand-in (Flan_1565 cannot be fetched)
        e = args.elements
        perm = False if args.permute < 0 else True if args.permute == 0 else args.permute
        return fa.elasticity_q1((e, e, e), contrast=1.0, nu=0.3, seed=42, permute=perm).upload(ctx)
    if args.problem == "mtx":  # a Matrix Market file placed on the box (e.g. Flan_1565.mtx)
        return fa.read_mtx(args.mtx).upload(ctx)
    raise ValueError(args.problem)


def build_problem(fa, ctx, args, dims):
    A = make_operator(fa, ctx, args, dims)
    if args.problem in ("7pt", "27pt"):
        mg = fa.sa_build_box(A, dims, (args.box,) * 3, coarsest_dim=1000, smoother=args.smoother)
    else:  # general SA: block size b, b constant-per-component candidates (C5)
        bs = args.block_size
        nn = fa.constant_candidates(A.nrows, bs)
        mg = fa.smoothed_aggregation(A, nn, block_size=bs, candidate_dimension=bs, coarsest_dim=1000,
                                     smoother=args.smoother, strength_depth=args.strength_depth)
    mg.set_reorder(args.reorder)
    return A, mg


def workload_name(args, dims):
    if args.problem in ("7pt", "27pt"):
        return (f"SA V-cycle, 3D {args.problem} {dims[0]}x{dims[1]}x{dims[2]}, box {args.box}^3, "
                f"{args.smoother} s=1 mu=1, Cholesky coarsest")
    perm = "all nodes" if args.permute == 0 else "no nodes" if args.permute < 0 else f"windows of {args.permute} nodes"
    src = (f"Q1 elasticity {args.elements}^3 elements (C5 stand-in: random E, node numbering shuffled "
           f"within {perm})"
           if args.problem == "elast" else f"Matrix Market {os.path.basename(args.mtx)}")
    return (f"SA V-cycle, {src}, block size {args.block_size}, {args.block_size} constant candidates, "
            f"strength graph depth {args.strength_depth} (reference: 3, partitioners/mod.rs:290), "
            f"MIS aggregates, block-Jacobi P smoothing, {args.smoother} s=1 mu=1, Cholesky coarsest")


def plan_summary(plan):
    """Per-level and whole-cycle algorithmic bytes from the library's own launch
    plan of one V-cycle (amg_multigrid_cycle_plan: every launch the cycle makes,
    with the bytes its storage streams and the vectors it moves).  Halo
    exchange records of a distributed plan (kernel -2) are summed apart
    (halo_bytes: what this rank sends + receives)."""
    lv = {}
    kern = [r for r in plan if r["kernel"] != -2]
    for r in plan:
        d = lv.setdefault(r["level"], {"launches": 0, "bytes": 0, "csr_bytes": 0, "halo_bytes": 0,
                                       "exchanges": 0, "kernels": []})
        if r["kernel"] == -2:
            d["halo_bytes"] += r["bytes"]
            d["exchanges"] += 1
            continue
        d["launches"] += 1
        d["bytes"] += r["bytes"]
        d["csr_bytes"] += r["csr_bytes"]
        d["kernels"].append(f"{r['role']}:{r['name']}:{r['mode']}")
    return {"launches": len(kern), "bytes": sum(r["bytes"] for r in kern),
            "csr_bytes": sum(r["csr_bytes"] for r in kern),
            "halo_bytes": sum(r["bytes"] for r in plan if r["kernel"] == -2),
            "per_level": [dict(level=l, **lv[l]) for l in sorted(lv)]}


def level_storages(mg):
    """Per level the storage of A_l, R_l, P_l (kernel, x-staged tile and how it
    was chosen: the frozen per-shape table of tuning.cpp or a setup-time timing),
    so two runs of one configuration can be compared decision by decision."""
    out = []
    for l in range(mg.levels()):
        Al, _, Rl, Pl = mg.level(l)
        d = {}
        for name, M in (("A", Al), ("R", Rl), ("P", Pl)):
            if M is None:
                continue
            i = M.spmv_info()
            e = {"kernel": i["kernel"], "gtc": i["gtc_kind"]}
            if i.get("xstaged"):
                e["tile"], e["tile_source"] = list(i["tile"]), i["tile_source"]
            d[name] = e
        out.append(d)
    return out


def abi_ingest(fa, ctx, mg, b, z_ref, stream, args):
    """The drop-in path's rate (what a Rust caller of INTEGRATION.md does): the
    hierarchy's arrays downloaded to the host and handed back level by level
    through amg_csr_create (no grid hints), new_jacobi / CoarseCholesky, then
    Multigrid::new + add_level (multigrid.rs:190-239, core.rs:56-74).  The same
    cycle is timed; z must equal the headline's bit for bit."""
    import numpy as np
    import torch
    t0 = time.perf_counter()
    nl = mg.levels()
    keep = []
    mg2 = None
    for l in range(nl):
        Al, Sl, Rl, Pl = mg.level(l)
        A2 = fa.SparseMatOp.from_arrays(ctx, *Al.dims(), *Al.arrays())
        if l == nl - 1:
            S2 = fa.CoarseCholesky(A2)
        elif Sl.kind == "sgs":
            S2 = fa.SymGaussSeidel(A2)
        elif Sl.kind == "diag" and args.smoother == "jacobi":
            S2 = fa.new_jacobi(A2, 0.66)
        elif Sl.kind == "diag" and args.smoother == "l1":
            S2 = fa.new_l1(A2)
        else:
            return {"skipped": f"no drop-in construction for the {Sl.kind} smoother"}
        if l == 0:
            mg2 = fa.Multigrid(A2, S2)
        else:
            R2 = fa.SparseMatOp.from_arrays(ctx, *Rp.dims(), *Rp.arrays())
            P2 = fa.SparseMatOp.from_arrays(ctx, *Pp.dims(), *Pp.arrays())
            mg2.add_level(A2, S2, R2, P2)
            keep += [R2, P2]
        keep += [A2, S2]
        Rp, Pp = Rl, Pl
    mg2.set_graph(not args.no_graph)
    mg2.set_fold_zero_guess(not args.no_fold)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    z2 = torch.empty_like(b)
    for _ in range(max(1, args.warmup)):
        mg2.apply(z2, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        mg2.apply(z2, b)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    same = bool(torch.equal(z2, z_ref))
    rel = float(torch.linalg.norm(z2 - z_ref) / torch.linalg.norm(z_ref))
    p1 = plan_summary(mg.cycle_plan())["per_level"]
    p2 = plan_summary(mg2.cycle_plan())["per_level"]
    kinds = [d["kernels"] for d in p2]
    grids = [mg2.level(l)[0].spmv_info()["grid_source"] for l in range(nl)]
    del mg2, keep
    torch.cuda.synchronize()
    return {"vcycles_per_s": round(1000.0 / ms, 3), "ms_per_step": round(ms, 4), "setup_s": round(setup_s, 2),
            "bitwise_equal_to_headline": same, "rel_diff": rel,
            "same_launch_plan": [d["kernels"] for d in p1] == kinds,
            "grid_hints": grids, "per_level_kernels": kinds,
            "what": "hierarchy arrays re-ingested through amg_csr_create + amg_multigrid_create/add_level "
                    "(no grid hints: inferred), same timed cycle as the headline"}


FUSED_NAMES = {0: ("fine-rr", "k_fine_rr",
                    "folded fine residual r = f - A (d f) + restriction f_c = R r, d_c f_c (r kept in LDS)"),
               1: ("fine-pj", "k_fine_pj",
                   "folded correction v = d f + P v_c + post-smoothing Jacobi step (v kept in LDS)")}


def fused_launches(mg, plan, b, z, stream, reps=20):
    """The cycle's fused fine-level launches (fine.hip) timed with HIP events on
    the library stream, priced on the algorithmic bytes of their plan records:
    inside the replayed V-cycle (events captured around the launch: the cache
    state the cycle gives it -- the headline figure), and alone, exactly as the
    V-cycle makes it on the cycle's own workspace (amg_multigrid_fine_launch):
    isolated_warm = the same rhs / out every launch, cold = rhs / out rotating
    over three pairs (a 1.6 GB working set, nothing MALL-resident)."""
    import numpy as np
    import torch
    out = {}
    recs = {p["name"]: p for p in plan if p["level"] == 0}
    for which, (pname, kname, what) in FUSED_NAMES.items():
        if pname not in recs or not mg.fine_launch(which, z, b):
            continue
        bytes_ = recs[pname]["bytes"]
        for _ in range(3):
            mg.fine_launch(which, z, b)
        warm = time_kernel(lambda: mg.fine_launch(which, z, b), reps, stream)
        pairs = [(b.clone(), torch.empty_like(z)) for _ in range(3)]
        it = [0]

        def rot():
            bb, zz = pairs[it[0] % 3]
            it[0] += 1
            mg.fine_launch(which, zz, bb)
        for _ in range(3):
            rot()
        cold = time_kernel(rot, 3 * reps, stream)
        del pairs
        torch.cuda.synchronize()
        # inside the V-cycle: HIP events around this launch (amg_multigrid_set_fine_timer;
        # the cycle's launches then run eagerly, the same kernels in the same order)
        mg.set_fine_timer(which)
        try:
            for _ in range(3):
                mg.apply(z, b)
            ins = []
            for _ in range(reps):
                mg.apply(z, b)
                ins.append(mg.fine_timer_ms())
        finally:
            mg.set_fine_timer(-1)
        inc = float(np.mean(ins))
        out[pname] = {"kernel": kname, "what": what, "bytes_per_launch": bytes_,
                      "csr_bytes_per_launch": recs[pname]["csr_bytes"],
                      "ms_per_launch": round(inc, 5), "achieved": round(bytes_ / (inc * 1e-3) / 1e9, 1),
                      "frac": round(bytes_ / (inc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "timing": (f"inside the V-cycle: HIP events around the launch in eager cycles (the "
                                 f"graph's kernels in the same order), mean of {reps} cycles (min {min(ins):.5f} ms)"),
                      "isolated_warm": {"ms_per_launch": round(warm, 5),
                                        "achieved": round(bytes_ / (warm * 1e-3) / 1e9, 1),
                                        "frac": round(bytes_ / (warm * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                        "what": "the launch alone, repeated on the same rhs / out"},
                      "cold": {"ms_per_launch": round(cold, 5),
                               "achieved": round(bytes_ / (cold * 1e-3) / 1e9, 1),
                               "frac": round(bytes_ / (cold * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                               "what": "the launch alone, rhs / out rotating over three pairs (1.6 GB > the 256 MB MALL)"}}
    return out


def fused_traffic(pname):
    """Calibrated PMC HBM bytes per launch of a fused fine-level kernel
    (scripts/pmc_cycle.sh -> profiles/rNN/c2_cycle_traffic.json, per plan
    position), or (None, None)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "c2_cycle_traffic.json")), reverse=True):
        d = json.load(open(f))
        for r in d.get("launches", []):
            if r.get("storage") == pname and r.get("hbm_bytes"):
                return r["hbm_bytes"], os.path.relpath(f, ROOT)
    return None, None


SECONDARY = (("c3_27pt_sgs", {"problem": "27pt", "smoother": "sgs"},
              "C3: 3D 27-point anisotropic 256^3, SA 2^3 boxes, multicolour SGS s=1, Cholesky coarsest"),
             ("c5_standin_shuffled", {"problem": "elast", "smoother": "l1", "permute": 4096},
              "C5 stand-in: Q1 elasticity 80^3 elements (1.57M rows), nodes shuffled within windows of 4096, "
              "general SA block 3, L1-Jacobi"),
             ("c5_standin_natural", {"problem": "elast", "smoother": "l1", "permute": -1},
              "C5 stand-in, the generator's lexicographic node numbering (no shuffle)"))


def secondary_one(fa, ctx, stream, a):
    """One secondary configuration on this GPU: setup, V-cycles/s of hipGraph
    replays (events on the library stream), the launch plan's bytes, and one
    V-cycle against the oracle on the same hierarchy."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    dims = (a.edge,) * 3
    t0 = time.perf_counter()
    A, mg = build_problem(fa, ctx, a, dims)
    mg.set_graph(True)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    n = A.nrows
    b_host = splitmix_uniform(n, 42)
    b = torch.as_tensor(b_host, device="cuda:0")
    z = torch.empty_like(b)
    for _ in range(3):
        mg.apply(z, b)
    ms = time_kernel(lambda: mg.apply(z, b), 20, stream)
    psum = plan_summary(mg.cycle_plan())
    t1 = time.perf_counter()
    omg = O.Multigrid(oracle_levels(mg, a.smoother))
    omg.set_parallel(a.cpu_threads)
    zref = omg.apply(b_host)
    rel = float(np.linalg.norm(z.cpu().numpy() - zref) / np.linalg.norm(zref))
    del omg
    res = {"vcycles_per_s": round(1000.0 / ms, 3), "ms_per_step": round(ms, 4), "steps": 20,
           "setup_s": round(setup_s, 2), "levels": mg.levels(), "fine_rows": n, "fine_nnz": A.nnz,
           "vcycle_launches": psum["launches"], "vcycle_algorithmic_GB": round(psum["bytes"] / 1e9, 3),
           "vcycle_GBs": round(psum["bytes"] / (ms * 1e-3) / 1e9, 1),
           "locality_renumbered_levels": [l for l in range(mg.levels()) if mg.reordered(l)],
           "parity": {"vcycle_rel_err": rel, "tol": 1e-11, "ok": rel <= 1e-11,
                      "oracle_s": round(time.perf_counter() - t1, 1),
                      "what": "one V-cycle z = M b (b = splitmix64 seed 42) against the oracle on the same hierarchy"}}
    del mg, A, b, z
    torch.cuda.synchronize()
    return res


def secondary_configs(fa, ctx, stream, args):
    """config.secondary: C3 and the C5 stand-in (both numberings) under the same
    clock as the headline, each with its own one-cycle oracle parity."""
    out = {}
    t_all = time.perf_counter()
    for name, over, what in SECONDARY:
        a = argparse.Namespace(**vars(args))
        for k, v in over.items():
            setattr(a, k, v)
        a.edge = 256
        t0 = time.perf_counter()
        try:
            out[name] = dict(secondary_one(fa, ctx, stream, a), workload=what)
        except Exception as e:  # reported, never fatal to the headline
            out[name] = {"error": repr(e), "workload": what}
        out[name]["wall_s"] = round(time.perf_counter() - t0, 1)
        log(f"secondary {name}: " + json.dumps({k: v for k, v in out[name].items() if k != "workload"}))
    out["wall_s"] = round(time.perf_counter() - t_all, 1)
    return out


def run_single(args):
    import numpy as np
    import torch

    import faer_amg_amd as fa

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(0, stream=stream.cuda_stream)
    dims = (args.edge,) * 3
    t0 = time.perf_counter()
    A, mg = build_problem(fa, ctx, args, dims)
    mg.set_graph(not args.no_graph)
    mg.set_fold_zero_guess(not args.no_fold)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    n = A.nrows
    levels = [{"n": mg.level(l)[0].nrows, "nnz": mg.level(l)[0].nnz} for l in range(mg.levels())]
    log(f"setup {setup_s:.2f}s levels={levels}")

    b_host = splitmix_uniform(n, 42)
    b = torch.as_tensor(b_host, device="cuda:0")
    z = torch.empty_like(b)
    for _ in range(args.warmup):
        mg.apply(z, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.trace_mark(1)  # k_trace_mark<<<1>>> ... <<<2>>> bracket the timed cycles in a kernel trace
    t_wall0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        mg.apply(z, b)
    e1.record(stream)
    ctx.trace_mark(2)
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t_wall0
    ms_per_cycle = e0.elapsed_time(e1) / args.steps

    # fine-level SpMV kernel (the one the V-cycle's fine smoothing/residual use),
    # timed with HIP events on the library stream
    # (a level-0 locality renumbering: the renumbered copy the cycle runs)
    x = torch.as_tensor(splitmix_uniform(n, 7), device="cuda:0")
    y = torch.empty_like(x)
    renumbered = mg.reordered(0)
    Arun = mg.run_level(0)[0] if renumbered else A
    for _ in range(3):
        Arun.apply(y, x)
    spmv_ms = time_kernel(lambda: Arun.apply(y, x), 20, stream)
    nnz = A.nnz
    info = Arun.spmv_info()
    bytes_spmv = spmv_bytes_fmt(Arun)
    del Arun
    bytes_csr = spmv_bytes(n, n, nnz)
    achieved = bytes_spmv / (spmv_ms * 1e-3) / 1e9

    # the same operator with fp64 values (value codes off): the uncompressed
    # SELL kernel, reported beside the one the V-cycle uses
    fa.set_value_codes(False)
    A64 = make_operator(fa, ctx, args, dims)
    fa.set_value_codes(True)
    for _ in range(3):
        A64.apply(y, x)
    spmv64_ms = time_kernel(lambda: A64.apply(y, x), 25, stream)  # 28 launches: apart from the cycle's in a trace
    bytes64 = spmv_bytes_fmt(A64)
    k64 = A64.spmv_info()["kernel"].replace("-", "_")
    fp64_values = {"kernel": f"spmv_{k64}_kernel<SET> on A_0, fp64 values", "ms_per_launch": round(spmv64_ms, 5),
                   "bytes_per_launch": bytes64,
                   "achieved": round(bytes64 / (spmv64_ms * 1e-3) / 1e9, 1),
                   "frac": round(bytes64 / (spmv64_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "storage": A64.spmv_info()}
    del A64

    general, csr_block = None, None
    if args.problem == "7pt" and not args.no_general:
        general = general_roofline(fa, ctx, dims, stream, x, y)
        log("roofline.general: " + json.dumps(general))
        csr_block = csr_roofline(general)

    if args.ab:
        ops = {}
        for fmt in ("csr", "sell"):
            fa.set_spmv_format(fmt)
            ops[fmt] = make_operator(fa, ctx, args, dims)
        fa.set_spmv_format("auto")
        res = {k: [] for k in ops}
        for _ in range(5):
            for fmt, op in ops.items():
                res[fmt].append(time_kernel(lambda: op.apply(y, x), 20, stream))
        for fmt, v in res.items():
            log(f"A/B fine SpMV {fmt}: median {np.median(v)*1e3:.1f} us  min {min(v)*1e3:.1f} us  "
                f"-> {spmv_bytes_fmt(ops[fmt]) / (min(v) * 1e-3) / 1e9:.0f} GB/s")
        del ops

    abi = None
    if not args.no_abi and args.problem in ("7pt", "27pt"):
        try:
            abi = abi_ingest(fa, ctx, mg, b, z, stream, args)
            log("abi ingest: " + json.dumps({k: v for k, v in abi.items() if k != "per_level_kernels"}))
        except Exception as e:  # reported, never fatal to the headline
            abi = {"error": repr(e)}
            log(f"abi ingest failed: {e!r}")

    r = torch.empty_like(b)
    A.apply(r, z)
    torch.cuda.synchronize()
    rho1 = float(torch.linalg.norm(b - r) / torch.linalg.norm(b))
    plan = mg.cycle_plan()
    psum = plan_summary(plan)
    storage_plan = level_storages(mg)
    vbytes, vbytes_csr = psum["bytes"], psum["csr_bytes"]
    if args.plan_out:
        with open(args.plan_out, "w") as fh:
            json.dump({"steps": args.steps, "plan": plan}, fh)

    # the cycle's fused fine-level launches timed on their own (roofline: the
    # dominant one -- the launch the V-cycle spends most time in)
    fused = {}
    if args.problem == "7pt" and not renumbered:
        zz = torch.empty_like(b)
        fused = fused_launches(mg, plan, b, zz, stream)
        del zz
        log("fused fine launches: " + json.dumps(fused))

    cpu, parity = None, None
    if not args.no_cpu_baseline:
        try:
            cpu, parity = cpu_side(mg, A, b_host, z.cpu().numpy(), args)
            log(f"parity: V-cycle rel err {parity['vcycle_rel_err']:.3e}, "
                f"rho_k max rel diff {parity['rho_k_max_rel_diff']:.3e}")
        except Exception as e:  # the baseline must not kill the GPU measurement
            log(f"cpu baseline / parity failed: {e!r}")

    secondary = None
    if args.problem == "7pt" and args.edge == 256 and not args.no_secondary:
        secondary = secondary_configs(fa, ctx, stream, args)

    cycles_per_s = 1000.0 / ms_per_cycle
    # (C5 stand-in: the counter file covers 80^3 elements, windows of 4096, renumbering on)
    c5_default = args.problem == "elast" and args.permute == 4096 and args.reorder == 1
    traffic, traffic_src = measured_traffic(args.elements if c5_default else args.edge, args.problem)
    # A_0's SET SpMV (the solve loops' operator apply); its CSR-equivalent rate
    # only where it stays below the HBM peak (a matrix-free stencil moves far
    # fewer bytes than CSR, so a CSR-priced rate above peak says nothing)
    csr_eq = bytes_csr / (spmv_ms * 1e-3) / 1e9
    a0_set = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
              "kernel": roofline_kernel_name(fa, info, args) + " on A_0"
                        + (" (locality-renumbered copy the cycle runs)" if renumbered else ""),
              "storage": info, "bytes_per_launch": bytes_spmv, "ms_per_launch": round(spmv_ms, 5),
              "csr_bytes_per_launch": bytes_csr}
    if csr_eq <= HBM_PEAK_GBS:
        a0_set["csr_equivalent_GBs"] = round(csr_eq, 1)
    else:
        a0_set["csr_equivalent_note"] = (f"CSR-priced rate {csr_eq / HBM_PEAK_GBS:.1f}x the HBM peak: the "
                                         f"storage streams {bytes_csr / bytes_spmv:.1f}x fewer bytes than CSR")
    if fused:
        # headline roofline: the cycle's dominant launch -- the fused fine-level
        # launch the V-cycle spends the most time in (measured here)
        dom = max(fused, key=lambda k: fused[k]["ms_per_launch"])
        f = fused[dom]
        ftraffic, fsrc = fused_traffic(dom)
        roofline = {"bound": "hbm", "achieved": f["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": f["frac"], "traffic": ftraffic, "traffic_source": fsrc,
                    "kernel": f"{f['kernel']} ({f['what']}) on level 0 -- the V-cycle's dominant launch",
                    "in_cycle": True, "timing": f["timing"], "bytes_per_launch": f["bytes_per_launch"],
                    "ms_per_launch": f["ms_per_launch"], "isolated_warm": f["isolated_warm"], "cold": f["cold"],
                    "fused": fused, "a0_set": a0_set, "fp64_values": fp64_values,
                    "csr": csr_block, "general": general}
    else:
        roofline = dict(a0_set, fp64_values=fp64_values, csr=csr_block, general=general)
    return {
        "metric": METRIC,
        "value": round(cycles_per_s, 3),
        "unit": "V-cycles/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_cycle, 4),
        "higher_is_better": True,
        "scaling": "none",
        "scaling_note": "single GPU: the N = 1 base of bench.py's default weak series "
                        "(256^3 rows per GPU fixed as N grows; --workload c4 gives the strong series)",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device-generated operator, splitmix64 rhs seed 42)",
        "config": {"workload": workload_name(args, dims),
                   "levels": len(levels), "fine_rows": n, "fine_nnz": nnz,
                   "hierarchy": levels, "setup_s": round(setup_s, 2),
                   "wall_ms_per_step": round(1000 * t_wall / args.steps, 4),
                   "vcycle_algorithmic_GB": round(vbytes / 1e9, 3),
                   "vcycle_GBs": round(vbytes / (ms_per_cycle * 1e-3) / 1e9, 1),
                   "vcycle_csr_equivalent_GB": round(vbytes_csr / 1e9, 3),
                   "vcycle_plan": {"launches": psum["launches"],
                                   "source": "amg_multigrid_cycle_plan (the launches the library makes)",
                                   "per_level_GB": [round(d["bytes"] / 1e9, 4) for d in psum["per_level"]],
                                   "per_level_launches": [d["launches"] for d in psum["per_level"]],
                                   "per_level_kernels": [d["kernels"] for d in psum["per_level"]],
                                   "per_level_storage": storage_plan},
                   "rel_residual_after_1_cycle": rho1,
                   "locality_renumbered_levels": [l for l in range(mg.levels()) if mg.reordered(l)],
                   "abi_ingest": abi,
                   "secondary": secondary,
                   "dense_tail": dense_tail_info(plan, levels),
                   "parallelism": "single GPU"},
        "fine_spmv_gbs": round(achieved, 1),
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity,
    }


def dense_tail_info(plan, levels):
    """The dense tail as the cycle ran it (ops.hip ensure_tail): the level whose
    launches down to the coarsest solve are one GEMV with the precomputed matrix
    of that part of the cycle, or None (every level launched)."""
    lt = max(p["level"] for p in plan)
    if lt >= len(levels) - 1:
        return None
    n = levels[lt]["n"]
    return {"level": lt, "rows": n, "matrix_bytes": 8 * n * n,
            "what": (f"levels {lt}..{len(levels) - 1} entered with v = 0 (mu = 1): that part of the cycle maps "
                     f"f_{lt} to v_{lt} linearly, so the cycle applies its {n} x {n} matrix (built once at the "
                     f"first apply by running it on the unit vectors) with one GEMV instead of its launches; "
                     f"the parity block compares against the oracle running every level")}


def roofline_kernel_name(fa, info, args):
    """The kernel A_0's SET launches (the name rocprofv3 reports for it)."""
    k = info["kernel"].replace("-", "_")
    if k == "dia" and args.problem == "7pt" and fa.get_flag("dia7_rp") in (0, 2):
        return "spmv_dia7c_kernel<SET, 2> (constant 7-point DIA, two row pairs per lane)"
    return f"spmv_{k}_kernel<SET>"


def run_dist(args, world, rank, local_rank):
    import numpy as np
    import torch
    import torch.distributed as dist

    import faer_amg_amd as fa

    dist.init_process_group("gloo")
    local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(local_rank, stream=stream.cuda_stream)
    strong = args.workload == "c4"
    dims = (512, 512, 512) if strong else weak_dims(args.edge, world)
    t0 = time.perf_counter()
    fa.set_spmv_format("csr")  # global (setup) copy: no SELL needed
    A, mg = build_problem(fa, ctx, args, dims)
    fa.set_spmv_format("auto")
    nl = mg.levels()
    if args.problem in ("7pt", "27pt"):
        splits = fa.slab_splits(fa.box_level_dims(dims, (args.box,) * 3, nl), world)
    else:  # equal row splits aligned to the level's block size
        splits = []
        for l in range(nl):
            n_l = mg.level(l)[0].nrows
            bs = args.block_size
            nb = n_l // bs
            splits.append([((p * nb) // world) * bs for p in range(world)] + [n_l])
    obj = [fa.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = fa.Comm(ctx, nranks=world, rank=rank, uid=obj[0])
    dm = fa.DistMultigrid(comm, mg, splits, agglomerate_rows=args.agglomerate).set_overlap(not args.no_overlap)
    infos = [dm.level_info(l) for l in range(nl)]
    La = sum(1 for i in infos if i["redundant"] == 0)

    def kind(M):
        i = M.spmv_info()
        k = "xscs" if i["kernel"] == "classes" and i["xstaged"] else i["kernel"]
        return k + ("+gtc" if i["gtc"] != "none" else "")
    storages = [{w: kind(dm.level_matrix(l, w)) for w in ("A", "R", "P")} for l in range(La)]
    n_glob = A_rows_global = A.nrows
    del mg, A  # global fine levels are no longer needed on this rank
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    log(f"rank {rank}: setup {setup_s:.1f}s, RCCL {fa.rccl_library()}, local storages {storages}")
    r0, r1 = dm.local_rows()
    b = torch.as_tensor(splitmix_uniform(n_glob, 42)[r0:r1].copy(), device=f"cuda:{local_rank}")
    z = torch.empty_like(b)
    raw_plan = dm.cycle_plan()  # collective: one eager cycle with the launch recorder on
    plan = plan_summary(raw_plan)
    if args.plan_out and rank == 0:
        with open(args.plan_out, "w") as fh:
            json.dump({"steps": args.steps, "plan": raw_plan}, fh)
    # hipGraph replay of the whole distributed cycle (RCCL p2p + all-gather
    # captured), checked bitwise against the eager cycle on every rank before it
    # is used; any difference or error falls back to the eager cycle
    graph = "off (--no-dist-graph)"
    if not args.no_dist_graph:
        ok, why = 1.0, ""
        try:
            ze, zg = torch.empty_like(b), torch.empty_like(b)
            dm.set_graph(False)
            dm.apply(ze, b)
            dm.set_graph(True)
            dm.apply(zg, b)  # capture + first replay
            dm.apply(zg, b)  # replay
            torch.cuda.synchronize()
            if not torch.equal(ze, zg):
                ok, why = 0.0, "replay differs from the eager cycle"
        except Exception as e:  # noqa: BLE001 -- reported in the line
            ok, why = 0.0, f"capture failed: {e!r}"
        t = torch.tensor([ok], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if float(t[0]) == 1.0:
            graph = "on (replay bitwise equal to the eager cycle on every rank)"
        else:
            dm.set_graph(False)
            graph = "eager fallback: " + (why or "another rank's replay check failed")
        log(f"rank {rank}: dist graph {graph}")
    for _ in range(args.warmup):
        dm.apply(z, b)
    torch.cuda.synchronize()
    dist.barrier()
    ctx.trace_mark(1)  # brackets the timed cycles in a kernel trace (scripts/prof_summary.py)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        dm.apply(z, b)
    torch.cuda.synchronize()
    el = time.perf_counter() - t_start
    ctx.trace_mark(2)
    dist.barrier()
    tmax = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    el = float(tmax[0])
    ms_per_cycle = 1000.0 * el / args.steps

    # local fine SpMV kernel on this rank (owned rows, [owned|ghost] columns)
    Al = dm.level_matrix(0, "A")
    nloc, ncl = Al.dims()
    xl = torch.as_tensor(splitmix_uniform(ncl, 7), device=f"cuda:{local_rank}")
    yl = torch.empty(nloc, dtype=torch.float64, device=f"cuda:{local_rank}")
    for _ in range(3):
        Al.apply(yl, xl)
    spmv_ms = time_kernel(lambda: Al.apply(yl, xl), 20, stream)
    al_info = Al.spmv_info()
    bytes_spmv = al_info["stream_bytes"] + 8 * nloc + 8 * nloc
    achieved = bytes_spmv / (spmv_ms * 1e-3) / 1e9
    # distributed fine SpMV including the halo exchange
    Ad = dm.level_operator(0)
    for _ in range(3):
        Ad.apply(yl, b)
    dist.barrier()
    halo_ms = time_kernel(lambda: Ad.apply(yl, b), 20, stream)

    # rho_k of the distributed stationary loop (collective) and the timed z gathered
    # on rank 0, for the parity checks below
    K = args.parity_cycles if args.parity_cycles is not None else (10 if A_rows_global <= (1 << 25) else 5)
    x = torch.zeros_like(b)
    it, hist = dm.stationary_solve(b, x, max_iter=K + 1, rel_tol=1e-300)
    hist = np.asarray(hist, np.float64)
    zparts = [None] * world if rank == 0 else None
    dist.gather_object((r0, z.cpu().numpy()), zparts, dst=0)
    ga = torch.tensor([achieved], dtype=torch.float64)
    dist.all_reduce(ga, op=dist.ReduceOp.MIN)
    cycles_per_s = 1000.0 / ms_per_cycle
    # rank 0, while the other ranks wait: the same global problem on this one GPU
    # (the single-GPU cycle the distributed one must reproduce; at 512^3 also
    # the base of the C4 strong-scaling ratio), then the oracle on that hierarchy
    # (parity of the distributed z and rho_k, and the CPU baseline)
    single, cpu, parity = None, None, None
    if rank == 0 and not args.no_single_base:
        del dm, Ad, Al
        torch.cuda.synchronize()
        try:
            z_dist = np.empty(A_rows_global)
            for (p0, zp) in zparts:
                z_dist[p0:p0 + zp.shape[0]] = zp
            single, cpu, parity = dist_single_side(fa, ctx, args, stream, dims, z_dist, hist)
        except Exception as e:  # reported, never fatal to the distributed measurement
            log(f"single-GPU base / parity failed: {e!r}")
            single = {"error": repr(e)}
    sb = torch.tensor([(single or {}).get("vcycles_per_s") or 0.0], dtype=torch.float64)
    dist.broadcast(sb, src=0)
    base = float(sb[0])
    ratio = round(cycles_per_s / base, 3) if base > 0 else None
    c4 = None
    if dims == (512, 512, 512) and args.problem == "7pt":
        c4 = {"global_vcycles_per_s": round(cycles_per_s, 3), "one_gpu_512_vcycles_per_s": round(base, 3),
              "ratio_vs_1gpu": ratio, "gpus": world,
              "what": "512^3 7-pt (C4): V-cycles/s of this row-split run / V-cycles/s of the same "
                      "hierarchy on one GPU (single-GPU path, measured in this job by rank 0)",
              "mall_caveat": C4_MALL_CAVEAT}
    out = dist_line(args, world, dims, strong, ms_per_cycle, cycles_per_s, ratio, c4, single, cpu, parity,
                    extra={"levels": nl, "level_plan_rank0": infos, "setup_s": round(setup_s, 2),
                           "fine_spmv_with_halo_ms": round(halo_ms, 4),
                           "rel_residual_after_1_cycle": float(hist[1]) if len(hist) > 1 else None,
                           "agglomerate_rows": args.agglomerate,
                           "halo_overlap": not args.no_overlap,
                           "dist_graph": graph,
                           "local_storages_rank0": storages,
                           "vcycle_plan_rank0": {"launches": plan["launches"],
                                                 "source": "amg_dist_cycle_plan (the launches this rank makes)",
                                                 "halo_bytes": plan["halo_bytes"],
                                                 "per_level_halo_bytes": [d["halo_bytes"] for d in plan["per_level"]],
                                                 "per_level_exchanges": [d["exchanges"] for d in plan["per_level"]],
                                                 "per_level_GB": [round(d["bytes"] / 1e9, 4)
                                                                  for d in plan["per_level"]],
                                                 "per_level_kernels": [d["kernels"] for d in plan["per_level"]]},
                           "rccl": fa.rccl_library(),
                           "rccl_ranks": comm.nranks},
                    roofline={"bound": "hbm", "achieved": round(float(ga[0]), 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(float(ga[0]) / HBM_PEAK_GBS, 4), "traffic": None,
                              "kernel": f"{al_info['kernel']} SpMV (SET) on the rank-local A_0 (min over ranks)",
                              "bytes_per_launch": bytes_spmv, "ms_per_launch": round(spmv_ms, 5)})
    dist.destroy_process_group()
    return out if rank == 0 else None


C4_MALL_CAVEAT = ("the one-GPU 512^3 base streams 1.07 GB vectors through a 256 MB MALL (cold), while each "
                  "rank of an N-GPU run holds a 256^3-sized slab whose vectors largely stay MALL-resident: "
                  "ratio_vs_1gpu can exceed N from cache alone; per_rank_vs_256cubed_single compares against "
                  "the MALL-warm 256^3 single-GPU rate instead")


DIST_LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "ratio_vs_1gpu", "ratio_vs_1gpu_what", "dtype", "data", "config",
                  "fine_spmv_gbs", "roofline", "cpu_baseline", "parity")


def dist_line(args, world, dims, strong, ms_per_cycle, cycles_per_s, ratio, c4, single, cpu, parity, extra,
              roofline, transport="RCCL"):
    """The JSON line of a distributed run (rank 0): value = global V-cycles/s (strong)
    or x N (weak: 256^3-equivalent cycles/s of the whole job); ratio_vs_1gpu = the
    global rate over the same global problem's one-GPU rate (at 512^3 the C4
    strong-scaling ratio); cpu_baseline / parity from the oracle on rank 0."""
    base256 = None
    if single:
        base256 = single.get("single_256_vcycles_per_s")
        if base256 is None and tuple(dims) == (256, 256, 256):
            base256 = single.get("vcycles_per_s")
    per_rank = (round(cycles_per_s * world / base256, 4)
                if cycles_per_s is not None and base256 and world > 1 else None)
    out = {
        "metric": METRIC,
        "value": None if cycles_per_s is None else round(cycles_per_s if strong else cycles_per_s * world, 3),
        "unit": "V-cycles/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None if ms_per_cycle is None else round(ms_per_cycle, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else ("weak" if world > 1 else "none"),
        "vs_baseline": None,
        "ratio_vs_1gpu": ratio,
        "ratio_vs_1gpu_what": (f"global V-cycles/s of this {world}-rank run / V-cycles/s of the same global "
                               f"problem ({dims[0]}x{dims[1]}x{dims[2]}) on one GPU, measured by rank 0 in this "
                               f"job" + (" = the C4 strong-scaling ratio (SURVEY.md 8(e), target >= 6 at 8 GPUs)"
                                         if tuple(dims) == (512, 512, 512) else "")),
        "dtype": "f64",
        "data": "synthetic (device-generated operator, splitmix64 rhs seed 42)",
        "config": dict({"workload": workload_name(args, dims) + (
                            f"; C4 strong scaling: fixed 512^3 over {world} ranks, value = global V-cycles/s"
                            if strong else f"; weak scaling: {world} x {args.edge}^3 rows, "
                                           f"value = global V-cycles/s x {world}"),
                        "c4_strong": c4,
                        "per_rank_vs_256cubed_single": per_rank,
                        "per_rank_vs_256cubed_single_what": (
                            f"global V-cycles/s x {world} / V-cycles/s of the 256^3 problem on one GPU "
                            f"({base256}, rank 0 in this job): per-GPU efficiency against a single GPU running "
                            f"the same 256^3-sized workload each rank holds -- the fair read of the weak "
                            f"series (both MALL-warm)"),
                        "single_gpu_same_problem": single,
                        "global_vcycles_per_s": None if cycles_per_s is None else round(cycles_per_s, 3),
                        "parallelism": f"row-block "
                                       f"{'z-slabs' if args.problem in ('7pt', '27pt') else 'row ranges'} "
                                       f"x{world}, {transport} halo exchange"}, **extra),
        "fine_spmv_gbs": roofline.get("achieved"),
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity,
    }
    assert tuple(out) == DIST_LINE_KEYS
    return out


def csr_roofline(general):
    """roofline.csr (verdict r04 item 1): the fine-level SpMV of a general CSR
    operator -- the 7-pt 256^3 graph with random coefficients (fp64 values, no
    value codes, no stencil structure) and rows shuffled within windows of 4096 --
    in the storage the auto policy gives it (x-staged SELL), priced on the bytes
    that storage moves per launch (format + x read once + y written) and on
    SURVEY.md 8(d)'s 32-bit CSR bytes; traffic = calibrated PMC HBM bytes of the
    same kernel (scripts/pmc_csr.sh)."""
    res = general["window4096"]
    kern = next(iter(res))  # the auto policy's storage (first entry)
    r = res[kern]
    moved, csr_b, ms = r["format_bytes_per_launch"], r["csr_bytes_per_launch"], r["ms_per_launch"]
    achieved = moved / (ms * 1e-3) / 1e9
    traffic, src = csr_traffic()
    return {"bound": "hbm", "kernel": f"{kern} SpMV (SET) on the random-coefficient 7-pt 256^3 operator, "
                                      f"rows shuffled within windows of 4096",
            "storage": kern, "ms_per_launch": ms,
            "bytes_per_launch": moved, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "csr_bytes_per_launch": csr_b, "csr_equivalent_GBs": r["achieved_csr_GBs"], "frac_csr": r["frac_csr"],
            "traffic": traffic, "traffic_source": src,
            "traffic_ratio": None if not traffic else round(traffic / moved, 4)}


def general_roofline(fa, ctx, dims, stream, x, y):
    """roofline.general: the fine SpMV on a matrix without stencil structure --
    the 7-pt graph with random edge weights (> 65536 distinct values: fp64
    values) and a symmetric row permutation (columns i32 / u16) -- in the SELL
    storage the auto policy picks and in CSR-stream, priced on SURVEY.md 8(d)'s
    CSR bytes (12 nnz + 4 (n+1) + 8 n + 8 n); the auto policy picks the x-staged
    SELL (xsell.hip) where each 4096-row group's x footprint fits LDS, SELL-64
    with u16/i32 columns otherwise.  Two permutations: within windows
    of 4096 rows (the locality of a mesh numbering) and over all rows (every x
    gather random)."""
    out = {}
    for name, window in (("window4096", 4096), ("random", 0)):
        res = {}
        for fmt in ("auto", "sell", "csr"):
            fa.set_spmv_format(fmt)
            try:
                M = fa.SparseMatOp.random7(ctx, *dims, seed=42, window=window)
            finally:
                fa.set_spmv_format("auto")
            for _ in range(3):
                M.apply(y, x)
            ms = time_kernel(lambda: M.apply(y, x), 20, stream)
            info = M.spmv_info()
            n, nnz = M.nrows, M.nnz
            csr_b = spmv_bytes(n, n, nnz)
            res[info["kernel"]] = {"ms_per_launch": round(ms, 5),
                                   "csr_bytes_per_launch": csr_b,
                                   "achieved_csr_GBs": round(csr_b / (ms * 1e-3) / 1e9, 1),
                                   "frac_csr": round(csr_b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "format_bytes_per_launch": info["stream_bytes"] + 16 * n,
                                   "storage": {k: info[k] for k in ("stream_bytes", "slices_u16", "slices_i32",
                                                                    "slices_implicit", "value_bits")}}
            del M
        out[name] = res
    return out


def dist_single_side(fa, ctx, args, stream, dims, z_dist, hist_dist, cycles=10):
    """Rank 0 of a distributed run, after its timing: the same global problem on
    this one GPU -- its V-cycles/s (at 512^3 the C4 base rate), its z against the
    distributed z (the row split keeps every row's arithmetic: <= 1e-13), then the
    oracle on that hierarchy: one cycle against the distributed z (<= 1e-11),
    rho_k of the distributed stationary loop against the oracle's (<= 1e-8), and
    the CPU baseline from the oracle's cycles (budgeted: at 512^3 one cycle of the
    restated rayon path takes seconds)."""
    A, mg = build_problem(fa, ctx, args, dims)
    out = single_side(fa, args, stream, A, mg, dims, z_dist, hist_dist, cycles)
    del mg, A
    import torch
    torch.cuda.synchronize()
    base256 = single_256_base(fa, ctx, args, stream, dims)
    if base256 and out[0] is not None and "error" not in out[0]:
        out[0]["single_256_vcycles_per_s"] = base256
    return out


def single_256_base(fa, ctx, args, stream, dims):
    """V-cycles/s of the 256^3 problem on this one GPU (the per-GPU workload of
    the weak series): the base of per_rank_vs_256cubed_single.  Skipped when the
    global problem is 256^3 itself (its single-GPU rate is that base)."""
    import torch
    if args.problem != "7pt" or tuple(dims) == (256, 256, 256):
        return None
    try:
        a = argparse.Namespace(**vars(args))
        a.edge = 256
        A, mg = build_problem(fa, ctx, a, (256, 256, 256))
        b = torch.as_tensor(splitmix_uniform(A.nrows, 42), device=torch.cuda.current_device())
        z = torch.empty_like(b)
        for _ in range(3):
            mg.apply(z, b)
        ms = time_kernel(lambda: mg.apply(z, b), 20, stream)
        del mg, A, b, z
        torch.cuda.synchronize()
        log(f"single-GPU 256^3 base: {1000.0 / ms:.1f} V-cycles/s")
        return round(1000.0 / ms, 3)
    except Exception as e:  # reported as missing, never fatal
        log(f"single-GPU 256^3 base failed: {e!r}")
        return None


def single_side(fa, args, stream, A, mg, dims, z_dist, hist_dist, cycles=10, what="the distributed GPU run"):
    """One-GPU rate of the global hierarchy (A, mg), its z against the distributed
    z, and the oracle's parity / CPU baseline on that hierarchy (dist_single_side)."""
    import numpy as np
    import torch
    n = A.nrows
    b_host = splitmix_uniform(n, 42)
    b = torch.as_tensor(b_host, device=torch.cuda.current_device())
    z = torch.empty_like(b)
    for _ in range(2):
        mg.apply(z, b)
    ms = time_kernel(lambda: mg.apply(z, b), cycles, stream)
    torch.cuda.synchronize()
    zs = z.cpu().numpy()
    rel = float(np.linalg.norm(z_dist - zs) / np.linalg.norm(zs))
    single = {"vcycles_per_s": round(1000.0 / ms, 3), "ms_per_step": round(ms, 4), "cycles": cycles,
              "z_rel_diff_vs_distributed": rel, "tol": 1e-13, "ok": rel <= 1e-13,
              "what": "the global problem's hierarchy on one GPU (single-GPU path) timed by rank 0 in this job; "
                      "its z = M b against the distributed run's timed z"}
    log(f"single-GPU base: {dims} {single['vcycles_per_s']:.2f} V-cycles/s, z rel diff vs distributed {rel:.2e}")
    cpu, parity = None, None
    if not args.no_cpu_baseline:
        K = len(hist_dist) - 1
        cpu, parity = cpu_side(mg, A, b_host, z_dist, args, hist_gpu=hist_dist, rho_cycles=K, min_cycles=1,
                               budget=args.cpu_budget / 2, what_gpu=what + " (z gathered on rank 0)")
        cpu["sample"] += f"; global problem {dims[0]}x{dims[1]}x{dims[2]}, rank 0's host"
        log(f"parity (distributed vs oracle): V-cycle rel err {parity['vcycle_rel_err']:.3e}, "
            f"rho_k max rel diff {parity['rho_k_max_rel_diff']:.3e} over {K} cycles")
    return single, cpu, parity


def run_loopback(args):
    """--loopback N: the distributed cycle with N virtual ranks on this one GPU
    (threads of this process over the library's loopback transport: the same
    row-block split, halo plans, slab frames and agglomeration as N RCCL ranks,
    with device copies instead of xGMI).  A rehearsal of the N-GPU line on a
    1-GPU box -- the same fields (parity against the oracle, CPU baseline,
    ratio to the one-GPU rate) -- whose rate measures N ranks time-sharing one
    GPU, not scaling."""
    import threading

    import numpy as np
    import torch

    import faer_amg_amd as fa

    N = args.loopback
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(0, stream=stream.cuda_stream)
    strong = args.workload == "c4"
    dims = (512, 512, 512) if strong else weak_dims(args.edge, N)
    t0 = time.perf_counter()
    A, mg = build_problem(fa, ctx, args, dims)
    n = A.nrows
    b_host = splitmix_uniform(n, 42)
    b = torch.as_tensor(b_host, device="cuda:0")
    zg = torch.empty_like(b)
    mg.apply(zg, b)  # codes the Jacobi diagonals before the ranks share the levels
    torch.cuda.synchronize()
    nl = mg.levels()
    splits = fa.slab_splits(fa.box_level_dims(dims, (args.box,) * 3, nl), N)
    hub = fa.LoopbackHub(N)
    comms, dms = [None] * N, [None] * N

    def ranks(fn):
        out, errs = [None] * N, []

        def body(r):
            try:
                out[r] = fn(r)
            except BaseException as e:  # noqa: BLE001
                errs.append(e)
        th = [threading.Thread(target=body, args=(r,)) for r in range(N)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return out

    def build(r):
        comms[r] = fa.Comm(ctx, hub=hub, rank=r)
        dms[r] = fa.DistMultigrid(comms[r], mg, splits, agglomerate_rows=args.agglomerate)
        return dms[r].local_rows()
    rows = ranks(build)
    setup_s = time.perf_counter() - t0
    infos = [dms[0].level_info(l) for l in range(nl)]
    bs = [b[r0:r1] for (r0, r1) in rows]
    zs = [torch.empty_like(bb) for bb in bs]
    for _ in range(args.warmup):
        ranks(lambda r: dms[r].apply(zs[r], bs[r]))
    torch.cuda.synchronize()

    def timed(r):
        for _ in range(args.steps):
            dms[r].apply(zs[r], bs[r])
    tw = time.perf_counter()
    ranks(timed)
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - tw) / args.steps
    K = args.parity_cycles if args.parity_cycles is not None else (10 if n <= (1 << 25) else 5)
    xs = [torch.zeros_like(bb) for bb in bs]
    hists = ranks(lambda r: dms[r].stationary_solve(bs[r], xs[r], max_iter=K + 1, rel_tol=1e-300)[1])
    z_dist = torch.cat(zs).cpu().numpy()
    del dms, comms
    torch.cuda.synchronize()
    single, cpu, parity = single_side(fa, args, stream, A, mg, dims, z_dist, np.asarray(hists[0]), 10,
                                      what=f"the {N}-rank loopback run")
    del mg, A
    torch.cuda.synchronize()
    base256 = single_256_base(fa, ctx, args, stream, dims)
    if base256:
        single["single_256_vcycles_per_s"] = base256
    cps = 1000.0 / ms
    ratio = round(cps / single["vcycles_per_s"], 3)
    c4 = None
    if dims == (512, 512, 512) and args.problem == "7pt":
        c4 = {"global_vcycles_per_s": round(cps, 3), "one_gpu_512_vcycles_per_s": single["vcycles_per_s"],
              "ratio_vs_1gpu": ratio, "gpus": 1, "virtual_ranks": N,
              "what": "loopback rehearsal: N virtual ranks time-share one GPU (not a scaling figure)",
              "mall_caveat": C4_MALL_CAVEAT}
    return dist_line(args, N, dims, strong, ms, cps, ratio, c4, single, cpu, parity,
                     extra={"levels": nl, "level_plan_rank0": infos, "setup_s": round(setup_s, 2),
                            "rel_residual_after_1_cycle": float(hists[0][1]) if len(hists[0]) > 1 else None,
                            "agglomerate_rows": args.agglomerate, "physical_gpus": 1,
                            "note": f"{N} virtual ranks on one GPU (loopback transport): value is not a "
                                    f"multi-GPU rate; the line rehearses the N-GPU line's fields"},
                     roofline={}, transport="loopback (device copies)")


def visible_gpus():
    """GPUs this process may use, counted without torch or HIP (the launcher
    stays provably GPU-free, so its children start on untouched devices): the
    *_VISIBLE_DEVICES lists when set, else the KFD topology's GPU nodes."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([t for t in v.split(",") if t.strip() and t.strip() != "-1"])
    import glob
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            kv = dict(line.split()[:2] for line in open(props) if len(line.split()) >= 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) > 0:  # CPU nodes have no SIMDs
            n += 1
    return n


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`python bench.py --gpus N` without an outer launcher: start N rank
    processes (torch.distributed.run, one per GPU, rendezvous on 127.0.0.1)
    as a child process, forward every rank's stderr and rank 0's JSON line,
    and return the exit status (non-zero when fewer than N GPUs are visible,
    a rank fails, or rank 0 printed no line)."""
    import subprocess
    if os.environ.get("FAMG_BENCH_LAUNCH_CHECK") != "1":
        have = visible_gpus()
        if have < n:
            log(f"bench.py --gpus {n}: only {have} GPU(s) visible")
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    env.setdefault("OMP_NUM_THREADS", "16")
    log("launching: " + " ".join(cmd))
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{"):
            try:
                d = json.loads(s)
            except ValueError:
                d = None
            if isinstance(d, dict) and "metric" in d:
                lines.append(s)
                continue
        sys.stderr.write(line)
    rc = proc.wait()
    if rc != 0:
        log(f"rank processes exited with status {rc}")
        return rc
    if len(lines) != 1:
        log(f"expected one JSON line from rank 0, got {len(lines)}")
        return 4
    print(lines[0], flush=True)
    return 0


def launch_check(world, rank):
    """FAMG_BENCH_LAUNCH_CHECK=1: what a rank does instead of the GPU work when
    the launcher is tested on a CPU-only machine -- join the process group
    (gloo), agree on the world size with an all-reduce, rank 0 returns a line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([1.0], dtype=torch.float64)
    dist.all_reduce(t)
    args = argparse.Namespace(steps=0, warmup=0, problem="7pt", edge=256, box=2, smoother="jacobi")
    world = dist.get_world_size()
    dims = weak_dims(256, world)
    out = dist_line(args, world, dims, False, None, None, None, None, None, None, None, {}, {})
    out.update({"ranks_counted": int(t[0]), "launch_check": True})
    dist.destroy_process_group()
    return out if rank == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--edge", type=int, default=256, help="grid edge per GPU")
    ap.add_argument("--box", type=int, default=2)
    ap.add_argument("--smoother", default=None, choices=["jacobi", "l1", "sgs", "block"],
                    help="default: jacobi (7pt), sgs (27pt), l1 (elast/mtx)")
    ap.add_argument("--problem", default="7pt", choices=["7pt", "27pt", "elast", "mtx"],
                    help="7pt (C2), 27pt (C3), elast (C5 stand-in), mtx (C5 with --mtx Flan_1565.mtx)")
    ap.add_argument("--elements", type=int, default=80, help="elast: elements per edge (80: 1.57M rows)")
    ap.add_argument("--mtx", default=None, help="mtx: path of a Matrix Market file")
    ap.add_argument("--permute", type=int, default=4096,
                    help="elast: node numbering shuffled within windows of this many nodes (the locality "
                         "of a mesh numbering without stencil structure); 0 = over all nodes; -1 = none "
                         "(the generator's lexicographic numbering)")
    ap.add_argument("--reorder", type=int, default=1, choices=[0, 1, 2],
                    help="locality renumbering of general levels (multigrid option 5): 0 off, 1 auto "
                         "(bitwise), 2 every eligible level")
    ap.add_argument("--block-size", type=int, default=3, help="elast/mtx: dofs per node")
    ap.add_argument("--strength-depth", type=int, default=1,
                    help="elast/mtx: BFS depth of the strength graph (the reference hard-codes 3, "
                         "partitioners/mod.rs:290; 1 by default here for memory, DESIGN.md 10)")
    ap.add_argument("--agglomerate", type=int, default=None,
                    help="levels with fewer global rows run redundantly on every rank "
                         "(default 16384 x world: a level is distributed while every rank owns "
                         ">= 16K of its rows; below that its halo exchanges cost more than the "
                         "redundant cycle)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-min-cycles", type=int, default=50,
                    help="CPU baseline: at least this many V-cycles at --cpu-threads")
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="seconds of CPU V-cycles at --cpu-threads (half that at all cores)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-dist-graph", action="store_true",
                    help="distributed: run the cycle eagerly instead of replaying it as a captured hipGraph "
                         "(RCCL p2p + all-gather captured; by default used after a bitwise check against the "
                         "eager cycle on every rank)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="distributed: exchange halos before the SpMV instead of under its interior rows")
    ap.add_argument("--ab", action="store_true", help="A/B the SpMV storage formats (stderr)")
    ap.add_argument("--no-general", action="store_true", help="skip roofline.general (random 7-pt)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip config.secondary (C3 and the C5 stand-in, both numberings, under the same clock)")
    ap.add_argument("--no-abi", action="store_true",
                    help="skip config.abi_ingest (the hierarchy re-ingested through the C ABI, timed)")
    ap.add_argument("--no-fold", action="store_true",
                    help="store the zero-guess smoothing step instead of folding it into the residual")
    ap.add_argument("--workload", default="weak", choices=["weak", "c4"],
                    help="N > 1: weak (N x edge^3 rows; at N = 8 the grid is 512^3 = C4 and the line "
                         "carries the C4 strong-scaling ratio) or c4 (512^3 fixed at every N, strong)")
    ap.add_argument("--no-single-base", "--no-c4-base", action="store_true",
                    help="distributed: skip rank 0's one-GPU run of the same global problem (the base of "
                         "ratio_vs_1gpu, at 512^3 the C4 ratio) and the parity / CPU baseline drawn from it")
    ap.add_argument("--parity-cycles", type=int, default=None,
                    help="distributed: stationary cycles compared with the oracle (default 10; 5 above 2^25 rows)")
    ap.add_argument("--plan-out", default=None,
                    help="write the V-cycle launch plan (JSON) here, for scripts/prof_summary.py --plan")
    ap.add_argument("--loopback", type=int, default=0,
                    help="N virtual ranks of the distributed cycle on this one GPU (loopback transport): "
                         "rehearses the N-GPU line's parity / CPU-baseline / ratio fields")
    ap.add_argument("--dist", action="store_true",
                    help="distributed path even at world size 1 (1-rank RCCL; a check of run_dist)")
    args = ap.parse_args()
    if args.agglomerate is None:
        args.agglomerate = 16384 * max(1, args.loopback, int(os.environ.get("WORLD_SIZE", "1")))
    if args.smoother is None:
        args.smoother = {"7pt": "jacobi", "27pt": "sgs"}.get(args.problem, "l1")
    if args.problem == "mtx" and not args.mtx:
        ap.error("--problem mtx needs --mtx PATH")

    if (args.gpus > 1 or args.dist) and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` (or --dist): start the N rank processes
        # ourselves (before anything touches the GPU) and forward rank 0's line
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus {args.gpus}; the job runs {world} ranks")
    if os.environ.get("FAMG_BENCH_LAUNCH_CHECK") == "1":
        out = launch_check(world, rank)  # CPU-only launcher check (tests/test_bench_launch.py)
        if out is not None:
            print(json.dumps(out), flush=True)
        return
    if args.workload == "c4" and world == 1 and not args.dist:
        args.edge = 512  # C4 on one GPU: the base of the strong-scaling curve
    if args.loopback > 0:
        out = run_loopback(args)
    elif world > 1 or args.dist:
        out = run_dist(args, world, rank, local_rank)
    else:
        out = run_single(args)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
