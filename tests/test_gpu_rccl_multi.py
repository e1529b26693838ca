"""Distributed hipGraph replay over a real RCCL communicator with N >= 2 ranks
(ADVICE r03): the captured cycle then holds the grouped ncclSend/ncclRecv on the
communication stream and its event fork/join.  Runs only where two GPUs are
visible (RCCL refuses two ranks on one GPU; the one-GPU boxes skip it and the
bench's own replay check covers the driver's 8-GPU runs)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _gpus():
    import torch
    return torch.cuda.device_count()  # counts without initialising the runtime on this image


@pytest.mark.timeout(600)
def test_rccl_two_rank_graph_replay_bitwise():
    n = min(_gpus(), 2)
    if n < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["FAMG_DENSE_TAIL"] = "0"  # the distributed cycle has no dense tail (ops.hip ensure_tail)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(HERE, "mgpu", "rccl_graph_check.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == n, p.stdout
    for r in lines:
        assert r["all_ranks_ok"] and r["overlap_True"] and r["overlap_False"] and r["overlap_neutral"], r
