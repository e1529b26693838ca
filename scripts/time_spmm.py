"""k-column SpMM against k single-vector SpMVs on the x-staged SELL and
pattern-SELL storages (verdict r05 item 8): ms per column, k in {8, 32}.
Writes gpurun_out/spmm_timing.json."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402


def ev_time(fn, reps):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = fa.Context(0, stream=stream.cuda_stream)
    dims = (256, 256, 256)
    mats = {"xsell random7 256^3 window 4096": fa.SparseMatOp.random7(ctx, *dims, seed=42, window=4096)}
    A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
    for l in range(mg.levels()):
        Al, _, Rl, Pl = mg.level(l)
        for nm, M in (("A", Al), ("R", Rl), ("P", Pl)):
            if M is not None and M.spmv_info()["kernel"] == "sellp":
                mats[f"sellp {nm}_{l} ({M.nrows} x {M.ncols})"] = M
    out = {}
    for name, M in mats.items():
        m, n = M.dims()
        res = {"kernel": M.spmv_info()["kernel"]}
        for k in (8, 32):
            X = torch.randn(k, n, dtype=torch.float64, device="cuda:0").t()
            Y = torch.empty(k, m, dtype=torch.float64, device="cuda:0").t()
            x1 = [X[:, c].contiguous() for c in range(k)]
            y1 = torch.empty(m, dtype=torch.float64, device="cuda:0")
            t_mm = ev_time(lambda: M.apply(Y, X), 5)

            def singles():
                for c in range(k):
                    M.apply(y1, x1[c])
            t_sv = ev_time(singles, 3)
            res[f"k{k}"] = {"spmm_ms_per_column": round(t_mm / k, 5), "spmv_ms_per_column": round(t_sv / k, 5),
                            "speedup": round(t_sv / t_mm, 2)}
        out[name] = res
        print(name, json.dumps(res), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "spmm_timing.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
