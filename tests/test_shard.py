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
