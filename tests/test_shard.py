"""Multi-process (gloo, world_size 2, CPU) coverage of the utterance-sharding path:
each rank runs its contiguous shard, rank 0 gathers; the result must equal the single-process one."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def test_shard_range_partitions():
    from sep_tfanet_vad_amd.shard import shard_range
    for n in (0, 1, 5, 64, 513):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (s0, e0), (s1, _) in zip(spans, spans[1:]):
                assert e0 == s1
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_path):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    from sep_tfanet_vad_amd.shard import gather_shards, run_shard
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234).items()}
    om = OracleModel(pkg.CONFIG_WITH_VAD, sd, torch.float64)
    x, _ = synth.make_batch(n, 4000, 900)
    sep_local = run_shard(lambda xs: om(xs)[0], torch.from_numpy(x), rank, world)
    full = gather_shards(sep_local, n)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_equal_single_process(tmp_path):
    import sys
    sys.path.insert(0, REPO)
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    n = 5  # ragged split: 3 + 2
    out = str(tmp_path / "sharded.npy")
    mp.spawn(_worker, args=(2, _free_port(), n, out), nprocs=2, join=True)
    sharded = np.load(out)
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234).items()}
    x, _ = synth.make_batch(n, 4000, 900)
    ref = OracleModel(pkg.CONFIG_WITH_VAD, sd, torch.float64)(torch.from_numpy(x))[0].numpy()
    assert sharded.shape == ref.shape
    assert np.abs(sharded - ref).max() <= 1e-12


def _bench_worker(rank, world, port, n, out_dir):
    """One rank of bench.py's own distributed path (init_dist / timed_region), gloo on CPU, with the
    oracle as the model and shard_range as the utterance split."""
    import sys
    import types
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import bench
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    from sep_tfanet_vad_amd.shard import shard_range
    d, w, r, lr = bench.init_dist(types.SimpleNamespace(gpus=world), backend="gloo")
    assert (w, r, lr) == (world, rank, rank) and d is not None
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234).items()}
    om = OracleModel(pkg.CONFIG_WITH_VAD, sd, torch.float32)
    x, _ = synth.make_batch(n, 4000, 901)
    s, e = shard_range(n, rank, world)
    xs = torch.from_numpy(x[s:e])
    outs = []

    def step():
        outs.append(om(xs)[0])

    el = bench.timed_region(step, 2, 1, d)
    np.save(os.path.join(out_dir, f"sep{rank}.npy"), outs[-1].numpy())
    np.save(os.path.join(out_dir, f"el{rank}.npy"), np.array([el, len(outs)]))
    d.barrier()
    d.destroy_process_group()


def test_bench_distributed_path_gloo(tmp_path):
    """bench.py's rank bookkeeping, barriers and max-over-ranks timing at world 2 (gloo): both ranks
    report the same (max) elapsed time, each ran warmup + steps forwards, and the shards concatenate
    to the single-process result."""
    import sys
    sys.path.insert(0, REPO)
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    n = 3
    mp.spawn(_bench_worker, args=(2, _free_port(), n, str(tmp_path)), nprocs=2, join=True)
    e0, e1 = np.load(tmp_path / "el0.npy"), np.load(tmp_path / "el1.npy")
    assert e0[0] == e1[0] > 0 and e0[1] == e1[1] == 3
    sharded = np.concatenate([np.load(tmp_path / "sep0.npy"), np.load(tmp_path / "sep1.npy")])
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234).items()}
    x, _ = synth.make_batch(n, 4000, 901)
    ref = OracleModel(pkg.CONFIG_WITH_VAD, sd, torch.float32)(torch.from_numpy(x))[0].numpy()
    assert np.abs(sharded - ref).max() <= 1e-6


def test_bench_launcher_only_outside_torchrun(monkeypatch):
    import sys
    import types
    sys.path.insert(0, REPO)
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_ranks(types.SimpleNamespace(gpus=2)) is None   # already a torchrun rank
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.launch_ranks(types.SimpleNamespace(gpus=1)) is None   # single GPU: in-process
    with pytest.raises(SystemExit):
        monkeypatch.setenv("WORLD_SIZE", "1")
        bench.init_dist(types.SimpleNamespace(gpus=2))                  # world must equal --gpus
