"""Benchmark: AMG V-cycle apply on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]

Step = one V-cycle (Multigrid::apply, multigrid.rs:469) of the smoothed-
aggregation hierarchy of the 3-D 7-point Laplacian, 256^3 per GPU (config
C2: 2^3 box aggregates, one constant candidate, weighted Jacobi omega=0.66,
s=1, mu=1, Cholesky coarsest), b ~ U(-1,1) from splitmix64 seed 42, x0 = 0.
Inputs are generated on the device and resident in HBM before timing.

Prints ONE JSON line on rank 0 (stdout); diagnostics go to stderr.
  value        V-cycles/s of the whole job (for N > 1: weak scaling, N z-slabs
               of 256^3 -> reported as 256^3-equivalent V-cycles/s)
  roofline     fine-level CSR SpMV kernel: algorithmic bytes / measured kernel
               time (HIP events on the library stream) vs 8 TB/s HBM peak
  cpu_baseline the oracle's restatement of the reference's rayon path
               (ParSpmmOp 8192x8192 CSC tiles, usize indices, per-call
               temporaries) on the same hierarchy, host threads stated
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def splitmix_uniform(n, seed=42):
    import numpy as np
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def spmv_bytes(nrows, ncols, nnz):
    """Algorithmic bytes of y = A x with 32-bit indices."""
    return 12 * nnz + 4 * (nrows + 1) + 8 * ncols + 8 * nrows


def time_kernel(fn, iters, stream):
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


def cpu_baseline(mg, b, threads, budget_s=12.0, max_cycles=40):
    """Reference-path restatement on the host (oracle ParSpmm + per-call temporaries)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    levels = []
    nl = mg.levels()
    for l in range(nl):
        Al, _, Rl, Pl = mg.level(l)
        d = {"A": O.Csr.from_arrays(*Al.dims(), *Al.arrays()),
             "smoother": "chol" if l == nl - 1 else "jacobi"}
        if Rl is not None:
            d["R"] = O.Csr.from_arrays(*Rl.dims(), *Rl.arrays())
            d["P"] = O.Csr.from_arrays(*Pl.dims(), *Pl.arrays())
        levels.append(d)
    omg = O.Multigrid(levels)
    omg.set_parallel(threads)
    out = np.empty_like(b)
    O.lib().orc_mg_apply(omg.h, b, out)  # warm-up (page faults)
    t0 = time.perf_counter()
    cycles = 0
    while cycles < max_cycles and (time.perf_counter() - t0) < budget_s:
        O.lib().orc_mg_apply(omg.h, b, out)
        cycles += 1
    dt = time.perf_counter() - t0
    return cycles / dt, cycles, dt, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=256, help="grid edge per GPU")
    ap.add_argument("--box", type=int, default=2)
    ap.add_argument("--smoother", default="jacobi", choices=["jacobi", "l1", "sgs"])
    ap.add_argument("--problem", default="7pt", choices=["7pt", "27pt"])
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch

    import faer_amg_amd as fa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 or args.gpus > 1:
        raise SystemExit("multi-GPU bench: see bench_dist (not yet wired)")

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(0, stream=stream.cuda_stream)
    nx = ny = nz = args.n
    t0 = time.perf_counter()
    if args.problem == "7pt":
        A = fa.SparseMatOp.laplace3d_7pt(ctx, nx, ny, nz)
    else:
        A = fa.SparseMatOp.aniso27(ctx, nx, ny, nz, 1.0, 1.0, 0.01)
    mg = fa.sa_build_box(A, (nx, ny, nz), (args.box,) * 3, coarsest_dim=1000,
                         smoother=args.smoother)
    mg.set_graph(not args.no_graph)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    n = A.nrows
    levels = []
    for l in range(mg.levels()):
        Al, _, _, _ = mg.level(l)
        levels.append({"n": Al.nrows, "nnz": Al.nnz})
    log(f"setup {setup_s:.2f}s levels={levels}")

    b_host = splitmix_uniform(n, 42)
    b = torch.as_tensor(b_host, device="cuda:0")
    z = torch.empty_like(b)
    for _ in range(args.warmup):
        mg.apply(z, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t_wall0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        mg.apply(z, b)
    e1.record(stream)
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t_wall0
    ms_per_cycle = e0.elapsed_time(e1) / args.steps
    cycles_per_s = 1000.0 / ms_per_cycle

    # fine-level SpMV kernel, timed on the library stream with HIP events
    x = torch.as_tensor(splitmix_uniform(n, 7), device="cuda:0")
    y = torch.empty_like(x)
    for _ in range(3):
        A.apply(y, x)
    spmv_ms = time_kernel(lambda: A.apply(y, x), 20, stream)
    nnz = A.nnz
    bytes_spmv = spmv_bytes(n, n, nnz)
    achieved = bytes_spmv / (spmv_ms * 1e-3) / 1e9

    # residual reduction of one V-cycle as a sanity figure
    r = torch.empty_like(b)
    A.apply(r, z)
    torch.cuda.synchronize()
    rho1 = float(torch.linalg.norm(b - r) / torch.linalg.norm(b))

    cpu = None
    if not args.no_cpu_baseline:
        try:
            v, cyc, dt, _ = cpu_baseline(mg, b_host, args.cpu_threads)
            cpu = {"value": round(v, 4), "unit": "V-cycles/s", "cores": args.cpu_threads,
                   "kind": "port",
                   "sample": f"{cyc} V-cycles of the same {nx}^3 hierarchy in {dt:.1f}s "
                             f"(oracle ParSpmmOp restatement, OpenMP {args.cpu_threads} threads)"}
        except Exception as e:  # baseline must not kill the GPU measurement
            log(f"cpu baseline failed: {e!r}")

    out = {
        "metric": "V-cycles/s + fine-level SpMV GB/s vs HBM peak, 3D 7-pt Laplacian 256³",
        "value": round(cycles_per_s, 3),
        "unit": "V-cycles/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_cycle, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device-generated 7-pt Laplacian, splitmix64 rhs seed 42)",
        "config": {"workload": f"SA V-cycle, 3D {args.problem} {nx}^3, box {args.box}^3, "
                               f"{args.smoother} s=1 mu=1, Cholesky coarsest",
                   "levels": len(levels), "fine_rows": n, "fine_nnz": nnz,
                   "hierarchy": levels, "setup_s": round(setup_s, 2),
                   "wall_ms_per_step": round(1000 * t_wall / args.steps, 4),
                   "rel_residual_after_1_cycle": rho1,
                   "parallelism": "single GPU"},
        "fine_spmv_gbs": round(achieved, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "kernel": "spmv_stream_kernel<SET> on A_0",
                     "bytes_per_launch": bytes_spmv, "ms_per_launch": round(spmv_ms, 5)},
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
