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
