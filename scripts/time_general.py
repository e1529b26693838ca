"""Time the fine SpMV of roofline.general (random 7-pt 256^3, rows shuffled in
windows of 4096) in the storage the auto policy picks: one line per run, for
A/B of env switches (e.g. FAMG_XS=0) in separate processes:
  FAMG_XS=0 python scripts/time_general.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import faer_amg_amd as fa  # noqa: E402
from bench import time_kernel, spmv_bytes  # noqa: E402

ctx = fa.Context(0)
stream = torch.cuda.current_stream()
dims = (256, 256, 256)
M = fa.SparseMatOp.random7(ctx, *dims, seed=42, window=int(os.environ.get("WINDOW", "4096")))
n = M.nrows
x = torch.rand(n, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
for _ in range(3):
    M.apply(y, x)
ms = time_kernel(lambda: M.apply(y, x), 30, stream)
info = M.spmv_info()
csr_b = spmv_bytes(n, n, M.nnz)
env = {k: v for k, v in os.environ.items() if k.startswith("FAMG_")}
print(f"{env} kernel={info['kernel']} ms={ms:.4f} frac_csr={csr_b / (ms * 1e-3) / 8e12:.4f} "
      f"format_GBs={(info['stream_bytes'] + 16 * n) / (ms * 1e-3) / 1e9:.0f}")
