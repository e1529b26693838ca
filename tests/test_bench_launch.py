"""bench.py --gpus N starts its own N rank processes (verdict r02 item 1).

The driver runs `python bench.py --gpus N` (and, for N > 1, possibly under an
outer torch.distributed.run).  Without WORLD_SIZE in the environment the
script must launch the ranks itself, before touching a GPU, and forward
exactly one JSON line from rank 0.  FAMG_BENCH_LAUNCH_CHECK=1 replaces each
rank's GPU work with a gloo all-reduce so the launcher runs on this CPU-only
machine."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks_and_forwards_one_line(n):
    p = run_bench(["--gpus", str(n), "--steps", "2", "--warmup", "1"], {"FAMG_BENCH_LAUNCH_CHECK": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["launch_check"] is True
    assert d["n_gpus"] == n and d["ranks_counted"] == n
    # a distributed line carries the one-GPU ratio, the CPU baseline and the
    # parity block beside the metric keys (bench.dist_line, verdict r04 item 2)
    import bench
    for k in bench.DIST_LINE_KEYS:
        assert k in d, k
    for k in ("ratio_vs_1gpu", "cpu_baseline", "parity", "roofline"):
        assert k in d
    assert d["scaling"] == "weak" and "single_gpu_same_problem" in d["config"]
    assert "per_rank_vs_256cubed_single" in d["config"]
    assert "torch.distributed.run" in p.stderr  # the launcher logged its child command


def test_launcher_refuses_without_enough_gpus():
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("machine has many GPUs")
    p = run_bench(["--gpus", "64", "--steps", "1", "--warmup", "0"], {}, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert p.stdout.strip() == ""
    assert "GPU(s) visible" in p.stderr


def test_launcher_counts_gpus_without_torch():
    """The launcher counts GPUs from *_VISIBLE_DEVICES / the KFD topology, never
    through torch or HIP (verdict r03: the parent must stay GPU-free)."""
    p = run_bench(["--gpus", "3", "--steps", "1", "--warmup", "0"],
                  {"HIP_VISIBLE_DEVICES": "0,1", "ROCR_VISIBLE_DEVICES": "0,1"}, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "only 2 GPU(s) visible" in p.stderr
    import bench
    src = __import__("inspect").getsource(bench.visible_gpus)
    assert "torch" not in src.split('"""')[2]


def test_dist_line_per_rank_vs_256cubed_single():
    """The N > 1 line's per-GPU efficiency against the MALL-warm 256^3 single-GPU
    rate (verdict r05 item 7): global V-cycles/s x N / the 256^3 one-GPU rate
    rank 0 measures; and the C4 block's MALL caveat text exists."""
    import argparse
    import bench
    args = argparse.Namespace(steps=5, warmup=1, problem="7pt", edge=256, box=2, smoother="jacobi")
    single = {"vcycles_per_s": 150.0, "single_256_vcycles_per_s": 1500.0}
    d = bench.dist_line(args, 8, (512, 512, 512), False, 5.0, 200.0, 1.33, None, single, None, None, {}, {})
    assert d["value"] == 1600.0
    assert abs(d["config"]["per_rank_vs_256cubed_single"] - 200.0 * 8 / 1500.0) < 1e-3
    assert "MALL" in bench.C4_MALL_CAVEAT
    d1 = bench.dist_line(args, 2, (256, 256, 512), False, 5.0, 700.0, 1.9, None, {"vcycles_per_s": 760.0},
                         None, None, {}, {})
    assert d1["config"]["per_rank_vs_256cubed_single"] is None  # no 256^3 base measured
