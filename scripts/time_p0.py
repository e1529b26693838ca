"""Time the fine-level transfer operators of the 256^3 hierarchy in SET mode
(y = M x) with HIP events, to compare with their in-cycle epilogues."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)
dims = (256,) * 3
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
_, _, R0, P0 = mg.level(0)


def timeit(op, x, y, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    op.apply(y, x)
    e0.record(stream)
    for _ in range(iters):
        op.apply(y, x)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for name, M in (("P0", P0), ("R0", R0)):
    m, n = M.dims()
    x = torch.rand(n, dtype=torch.float64, device="cuda:0")
    y = torch.empty(m, dtype=torch.float64, device="cuda:0")
    info = M.spmv_info()
    t = min(timeit(M, x, y) for _ in range(5))
    print(f"{name} {m}x{n} {info['kernel']} vb={info['value_bits']} stream={info['stream_bytes']/1e6:.1f}MB SET {t:.1f} us "
          f"({(info['stream_bytes'] + 8 * n + 8 * m) / (t * 1e-6) / 1e12:.2f} TB/s incl. x once + y)", flush=True)
