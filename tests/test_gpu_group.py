"""Heterogeneous batches (mbik_group_*): distinct rigs solved by one launch, each bitwise equal
to the oracle and to its own plan's solve."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Group, Plan

from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def rigs():
    two_roots = W.custom_topology([-1, -1, 1, -1, 3, 4], [2, 5], [4, 5], cones_per_bone=1, twist=(0.1, 1.0),
                                  iterations=5)
    return [
        (W.generate(2, 96), dict()),
        (W.generate(5, 6), dict()),
        (W.generate(14, 40, topo=two_roots), dict(lanes=4)),
        (W.generate(2, 24, first=500), dict(stabilization_passes=1)),
        (W.generate(3, 64), dict(lanes=2)),
    ]


def upload(torch, dev, wl):
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    return pi, tg, torch.empty_like(pi)


def test_group_matches_oracle(oracle, mbik, torch_dev):
    torch, dev = torch_dev
    cases = rigs()
    plans = [Plan.from_workload(wl, **kw) for wl, kw in cases]
    bufs = [upload(torch, dev, wl) for wl, _ in cases]
    g = Group(plans)
    g.solve([b[0].data_ptr() for b in bufs], [b[1].data_ptr() for b in bufs], [b[2].data_ptr() for b in bufs])
    torch.cuda.synchronize()
    for (wl, kw), b in zip(cases, bufs):
        ref = oracle.Oracle(wl, stabilization_passes=kw.get("stabilization_passes", 0)).solve(wl.pose, wl.targets, threads=4)
        assert_parity(b[2].cpu().numpy(), ref, f"{wl.topo.name}")
    g.close()


def test_group_subranges_and_repeat(oracle, mbik, torch_dev):
    """Per-plan skeleton ranges; two frames on one stream reuse the group's tables."""
    torch, dev = torch_dev
    cases = rigs()[:3]
    plans = [Plan.from_workload(wl, **kw) for wl, kw in cases]
    g = Group(plans)
    first = [5, 1, 10]
    count = [40, 3, 0]
    subs = []
    for (wl, _), f, c in zip(cases, first, count):
        sub_pose = np.ascontiguousarray(wl.pose[f:f + c])
        sub_tg = np.ascontiguousarray(wl.targets[f:f + c])
        subs.append((torch.from_numpy(sub_pose).to(dev), torch.from_numpy(sub_tg).to(dev)))
    outs = [torch.full_like(s[0], float("nan")) for s in subs]
    for _ in range(2):
        g.solve([s[0].data_ptr() for s in subs], [s[1].data_ptr() for s in subs], [o.data_ptr() for o in outs],
                first=first, count=count)
    torch.cuda.synchronize()
    for (wl, kw), f, c, o, p in zip(cases, first, count, outs, plans):
        if c == 0:
            assert torch.isnan(o).all()     # untouched
            continue
        ref = p.solve_host(wl.pose[f:f + c], wl.targets[f:f + c], first=f)
        assert_parity(o.cpu().numpy(), ref, f"{wl.topo.name} [{f}, {f + c})")
    g.close()


def test_group_with_constraint_mode_and_pinless(oracle, mbik, torch_dev):
    torch, dev = torch_dev
    wl_c = W.generate(2, 16)
    wl_n = W.generate(13, 4, topo=W.custom_topology([-1, 0, 1], [], []))
    wl_d = W.generate(2, 32)
    plans = [Plan.from_workload(wl_c, constraint_mode=True), Plan.from_workload(wl_n), Plan.from_workload(wl_d)]
    bufs = [upload(torch, dev, w) for w in (wl_c, wl_n, wl_d)]
    g = Group(plans)
    g.solve([b[0].data_ptr() for b in bufs], [b[1].data_ptr() for b in bufs], [b[2].data_ptr() for b in bufs])
    torch.cuda.synchronize()
    assert_parity(bufs[0][2].cpu().numpy(), oracle.Oracle(wl_c, constraint_mode=True).solve(wl_c.pose, wl_c.targets), "cmode")
    assert np.array_equal(bufs[1][2].cpu().numpy(), wl_n.pose)
    assert_parity(bufs[2][2].cpu().numpy(), oracle.Oracle(wl_d).solve(wl_d.pose, wl_d.targets), "default")
    g.close()
