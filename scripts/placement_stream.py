"""Placement effect on plain streaming reads: several 1.34 GB buffers (the size
of the 256^3 7-pt SELL record array) with unrelated allocations in between,
each summed by torch in interleaved rounds.  If read bandwidth varies per
buffer the SpMV placement effect is a memory-system property, not the kernel's."""
import torch

GB = 1341 * 1024 * 1024
bufs, pads = [], []
for k in range(8):
    bufs.append(torch.rand(GB // 8, dtype=torch.float64, device="cuda:0"))
    pads.append(torch.empty((k + 1) * 37 * 1024 * 1024 + 12345, dtype=torch.uint8, device="cuda:0"))
out = torch.empty(1, dtype=torch.float64, device="cuda:0")


def t(b, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.sum(b, dim=0, out=out)
    e0.record()
    for _ in range(it):
        torch.sum(b, dim=0, out=out)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


res = {}
for r in range(5):
    for i, b in enumerate(bufs):
        res.setdefault(i, []).append(t(b))
for k, v in sorted(res.items()):
    us = sorted(v)[2]
    print(f"buffer {k} {bufs[k].data_ptr():#x}: median {us:7.1f} us  {GB / us / 1e3:7.1f} GB/s")
