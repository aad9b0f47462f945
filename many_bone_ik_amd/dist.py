"""Multi-GPU sharding of a skeleton batch.

Skeletons are independent, so rank r of W owns the contiguous range
[r*N/W, (r+1)*N/W) and solves it with no collective on the data path.  The only
exchange is the final gather of output poses (RCCL all_gather over xGMI with the
"nccl" backend; "gloo" on CPU for tests).
"""
from __future__ import annotations


def shard_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """(first, count) of this rank's contiguous share; the first total % world ranks get one more."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def gather_poses(pose_out, total: int, group=None):
    """All-gather every rank's [count, B, 10] pose shard into a [total, B, 10] tensor.

    Shards may differ by one skeleton; they are padded to the largest shard for the
    collective (one all_gather call, fixed message size) and trimmed afterwards.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_range(r, world, total)[1] for r in range(world)]
    cmax = max(counts)
    pad = pose_out
    if pose_out.shape[0] < cmax:
        pad = torch.zeros((cmax,) + tuple(pose_out.shape[1:]), dtype=pose_out.dtype, device=pose_out.device)
        pad[: pose_out.shape[0]] = pose_out
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    assert counts[rank] == pose_out.shape[0]
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)


def gather_poses_to_root(pose_out, total: int, root: int = 0, group=None):
    """Gather every rank's pose shard onto `root` only (the ranks send, the
    root receives world-1 shards, one per xGMI link in parallel -- RCCL send/recv under the
    "nccl" backend).  Returns the [total, B, 10] tensor on `root`, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_range(r, world, total)[1] for r in range(world)]
    cmax = max(counts)
    assert counts[rank] == pose_out.shape[0]
    pad = pose_out
    if pose_out.shape[0] < cmax:
        pad = torch.zeros((cmax,) + tuple(pose_out.shape[1:]), dtype=pose_out.dtype, device=pose_out.device)
        pad[: pose_out.shape[0]] = pose_out
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == root else None
    dist.gather(pad, gather_list=parts, dst=root, group=group)
    if rank != root:
        return None
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
