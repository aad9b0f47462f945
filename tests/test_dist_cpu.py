"""N>1 path on CPU: world_size-2 gloo, contiguous skeleton shards solved independently and
gathered (the GPU bench uses the same shard_range / gather_poses over RCCL)."""
import os

import numpy as np
import pytest

from many_bone_ik_amd.dist import shard_range


def test_shard_range_partitions():
    for total in [0, 1, 7, 4096, 4097]:
        for world in [1, 2, 3, 8]:
            seen = []
            for r in range(world):
                f, c = shard_range(r, world, total)
                seen.extend(range(f, f + c))
            assert seen == list(range(total))


def _worker(rank, world, port, total, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from many_bone_ik_amd import workloads as W
    from many_bone_ik_amd.dist import gather_poses, gather_poses_to_root
    from oracle import pyoracle as po
    first, count = shard_range(rank, world, total)
    wl = W.generate(2, count, first=first)
    out = po.Oracle(wl).solve(wl.pose, wl.targets)      # CPU stand-in for the per-rank solve
    full = gather_poses(torch.from_numpy(out), total)
    rooted = gather_poses_to_root(torch.from_numpy(out), total, root=world - 1)
    assert (rooted is None) == (rank != world - 1)
    if rank == world - 1:
        assert np.array_equal(rooted.numpy().view(np.uint32), full.numpy().view(np.uint32))
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.destroy_process_group()


def test_gloo_world2_shard_and_gather(oracle, tmp_path):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    total = 7
    out_path = str(tmp_path / "gathered.npy")
    mp.spawn(_worker, args=(2, port, total, out_path), nprocs=2, join=True)
    from many_bone_ik_amd import workloads as W
    wl = W.generate(2, total)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets)
    got = np.load(out_path)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
