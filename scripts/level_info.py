"""Print the SpMV storage of every operator of the bench hierarchy (A_l, R_l, P_l):
kernel, stream bytes, value-code bits and table size.  GPU box only.

  python scripts/level_info.py [--edge 256] [--problem 7pt|27pt]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edge", type=int, default=256)
    ap.add_argument("--problem", choices=("7pt", "27pt"), default="7pt")
    args = ap.parse_args()
    ctx = fa.Context()
    dims = (args.edge,) * 3
    if args.problem == "7pt":
        A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
        mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000, smoother="jacobi")
    else:
        A = fa.SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
        mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000, smoother="sgs")
    for l in range(mg.levels()):
        a, _, r, p = mg.level(l)
        for name, M in (("A", a), ("R", r), ("P", p)):
            if M is None:
                continue
            info = M.spmv_info()
            info.update(level=l, op=name, nrows=M.nrows, ncols=M.ncols, nnz=M.nnz)
            print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
