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


def _bench(*args, env=None):
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(here, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=e, cwd=here)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("scaling,total", [("weak", 2 * 7), ("strong", 7)])
def test_bench_launches_its_own_ranks(scaling, total):
    """`bench.py --gpus 2` as a plain command (how the driver's scaling run may call it) starts
    torch.distributed.run itself; the line reports n_gpus == --gpus and the gathered shards
    cover the batch in order (dry run: gloo, no GPU, no solve)."""
    rc, line, err = _bench("--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--skeletons", "7",
                           "--scaling", scaling)
    assert rc == 0, err[-2000:]
    assert line["dry_run"] and line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["config"]["skeletons_total"] == total
    assert line["gathered_in_order"]
    # the gathers report what they move: skeletons of [1, 10] floats, shards padded to the larger
    g = line["gather"]
    shard = (total + 1) // 2 * 10 * 4
    assert g["pose_bytes_total"] == total * 40 and g["shard_bytes_padded"] == shard
    assert g["all_gather"]["bytes_in_per_rank"] == shard and g["all_gather"]["ms"] > 0
    assert g["all_gather"]["GBps_in_per_rank"] > 0
    assert g["to_root"]["bytes_in_root"] == shard and g["to_root"]["GBps_in_root"] > 0


def test_bench_refuses_world_mismatch():
    rc, line, err = _bench("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and line is None
    assert "one rank per GPU" in err
