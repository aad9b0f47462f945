"""GPU-side plan build: the topology builder on the device (one thread per
rig) equals the host builder table for table, and a crowd of distinct rigs whose topologies and
setup frames were built only on the GPU (mbik_plan_create_device) solves in one fused launch
bitwise like the oracle."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Group, Plan, plans_from_device, topology_selftest

from .test_gpu_parity import assert_parity
from .test_topology_build import all_rigs, rig_of_workload

pytestmark = pytest.mark.gpu

CROWD_EDGE = {
    "dropped_branch": ([-1, 0, 1, 1, 3, 0, 5, 6], [2, 7], [1, 2, 5, 6, 7], 2, (0.2, 1.5)),
    "multi_root_released_origin": ([-1, 0, 1, -1, 3, 4], [2, 5], [1, 2, 4, 5], 1, (-0.3, 2.0)),
    "pinned_root": ([-1, 0, 1, 0, 3], [0, 2, 4], [1, 2, 3, 4], 2, (0.0, math.tau)),
    "unsorted_parents": ([2, 2, -1, 1, 0], [3, 4], [0, 1, 3, 4], 2, (0.0, 1.0)),
    "wide_fan_17_effectors": ([-1] + [0] * 17 + list(range(1, 18)), list(range(18, 35)), [], 0, None),
}


def test_device_topology_builder_equals_host_builder(mbik):
    rigs = all_rigs()
    mism, err = topology_selftest(rigs, device=0)
    bad = [i for i, m in enumerate(mism) if m]
    assert not bad, f"rigs {bad[:10]} differ: {err}"


def _crowd():
    wls = [W.generate(2, 32, first=11), W.generate(5, 4, first=3), W.generate(3, 16, first=70), W.generate(4, 6, first=5)]
    for k, (name, (parents, pins, cons, nc, twist)) in enumerate(CROWD_EDGE.items()):
        wls.append(W.generate(20 + k, 8, topo=W.custom_topology(parents, pins, cons, cones_per_bone=nc, twist=twist)))
    return wls


def test_crowd_built_on_the_device_solves_bitwise(oracle, mbik):
    import torch
    dev = torch.device("cuda", 0)
    wls = _crowd()
    keep = []

    def up(a):
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        keep.append(t)
        return t.data_ptr()

    rigs = [rig_of_workload(wl) for wl in wls]
    has_c = [wl.topo.constrained.shape[0] > 0 for wl in wls]
    plans = plans_from_device(rigs, [wl.n for wl in wls], [up(wl.pose) for wl in wls],
                              [up(wl.cones) if c else 0 for wl, c in zip(wls, has_c)],
                              [up(wl.twist) if c else 0 for wl, c in zip(wls, has_c)])
    # the GPU-built setup frames equal the host builder's
    for wl, p in zip(wls, plans):
        host = Plan.from_workload(wl)
        for a, b in zip(p.setup_tables(), host.setup_tables()):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
        host.close()
    grp = Group(plans)
    pin = [up(wl.pose) for wl in wls]
    tg = [up(wl.targets) for wl in wls]
    outs = [torch.empty_like(torch.from_numpy(wl.pose)).to(dev) for wl in wls]
    grp.solve(pin, tg, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for k, (wl, o) in enumerate(zip(wls, outs)):
        ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
        assert_parity(o.cpu().numpy(), ref, f"device-built rig {k}")


def test_device_plans_refuse_bad_rigs(mbik):
    import torch
    from many_bone_ik_amd import _lib
    pose = torch.zeros((1, 2, 10), device="cuda:0")
    with pytest.raises(_lib.MbikError) as e:
        plans_from_device([(np.array([1, 0], np.int32), [dict(bone=0)], [], {})], [1], [pose.data_ptr()])
    assert e.value.code == _lib.MBIK_EINVAL and "cycle" in str(e.value)


def test_device_plans_bad_rig_after_good_leaks_nothing(mbik):
    """A crowd whose second rig is refused (more cones than max_cones) fails as a whole, before
    the first rig's plan takes device memory: repeating the call frees as much as it took."""
    import torch
    from many_bone_ik_amd import _lib
    dev = torch.device("cuda", 0)
    wl = W.generate(5, 2048)                       # ~130 MB of setup tables per good plan
    keep = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (wl.pose, wl.cones, wl.twist)]
    bad_pose = torch.zeros((1, 2, 10), device=dev)
    bad_cones = torch.zeros((1, 1, 3, 4), device=dev)
    bad_twist = torch.zeros((1, 1, 3), device=dev)
    bad = (np.array([-1, 0], np.int32), [dict(bone=1)], [dict(bone=1, cone_count=3)], {"max_cones": 1})
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    for _ in range(4):
        with pytest.raises(_lib.MbikError) as e:
            plans_from_device([rig_of_workload(wl), bad], [wl.n, 1], [keep[0].data_ptr(), bad_pose.data_ptr()],
                              [keep[1].data_ptr(), bad_cones.data_ptr()], [keep[2].data_ptr(), bad_twist.data_ptr()])
        assert e.value.code == _lib.MBIK_EINVAL and "rig 1" in str(e.value)
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info(0)[0] >= free0 - (64 << 20)


def test_device_builder_on_a_large_random_crowd(mbik):
    """2,048 random rigs (random trees, pins, priorities, weights, propagation factors,
    constraints, damping, stabilization) built in one launch: every table as the host's."""
    from .test_topology_build import random_rig
    rigs = [random_rig(10_000 + s) for s in range(2048)]
    mism, err = topology_selftest(rigs, device=0)
    assert not any(mism), err
