"""bench.py output contract on the GPU: stdout is exactly one JSON line carrying the driver's keys plus
the roofline object; the measured path is the native library (no CPU leg with --no-cpu-baseline)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline"}
ROOF = {"bound", "achieved", "peak", "unit", "frac", "traffic"}


def test_bench_prints_one_json_line():
    p = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                       cwd=REPO, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[:2000]
    d = json.loads(lines[0])
    assert KEYS <= d.keys()
    assert ROOF <= d["roofline"].keys()
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 64 and d["config"]["seq_len"] == 32000
    r = d["roofline"]
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3


def test_bench_rccl_path_one_json_line():
    """The multi-GPU timing path (process group over RCCL, barrier + max-reduce around the timed region) under
    torch.distributed.run, forced at world 1 on a one-GPU box: still exactly one JSON line on stdout even though
    RCCL prints its banner to fd 1 on some hosts (bench.py hold_stdout)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, SEPVAD_BENCH_FORCE_DIST="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                       cwd=REPO, capture_output=True, text=True, timeout=150, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[:2000]
    d = json.loads(lines[0])
    assert KEYS <= d.keys() and d["n_gpus"] == 1 and d["value"] > 0


def _one_json(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[:2000]
    return json.loads(lines[0])


def test_bench_two_ranks_through_the_launcher():
    """bench.py --gpus 2 outside torchrun: launch_ranks starts a child torch.distributed.run with two ranks (here both
    on cuda:0 over gloo, SEPVAD_BENCH_SHARE_GPU=1: RCCL needs a GPU per rank); exactly one JSON line from rank 0 with
    the whole-job numbers. Two persistent k_tcn grids share the chip and both finish (no cooperative launch)."""
    env = dict(os.environ, SEPVAD_BENCH_SHARE_GPU="1")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                       cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    d = _one_json(p)
    assert KEYS <= d.keys()
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 128 and d["value"] > 0


def test_bench_stream_two_ranks_equal_one_rank(tmp_path):
    """cfg 3 sharded over two ranks (256 streams each, the PIT-L1 sums all-reduced: model/pit_wrapper.py:172-177 is
    batch-global) equals one rank running all 512 streams, bitwise (stream inputs are seeded per stream)."""
    env2 = dict(os.environ, SEPVAD_BENCH_SHARE_GPU="1", SEPVAD_BENCH_DUMP=str(tmp_path / "w2"))
    p2 = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--workload", "stream", "--steps", "1", "--warmup",
                         "0", "--no-cpu-baseline"], cwd=REPO, capture_output=True, text=True, timeout=280, env=env2)
    d2 = _one_json(p2)
    assert d2["n_gpus"] == 2 and d2["config"]["global_batch"] == 512
    env1 = dict(os.environ, SEPVAD_BENCH_DUMP=str(tmp_path / "w1"))
    p1 = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--workload", "stream", "--batch", "512",
                         "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], cwd=REPO, capture_output=True, text=True,
                        timeout=280, env=env1)
    _one_json(p1)
    import numpy as np
    a = np.concatenate([np.load(str(tmp_path / "w2.rank0.npy")), np.load(str(tmp_path / "w2.rank1.npy"))])
    b = np.load(str(tmp_path / "w1.rank0.npy"))
    assert a.shape == b.shape == (512, 2, 7 * 2560)
    assert np.isfinite(a).all()
    assert np.array_equal(a, b)
