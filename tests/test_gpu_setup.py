"""GPU plan setup (mbik_plan_rebuild_setup): the per-skeleton bone-direction
and Kusudama frames derived on the device equal the host builder's tables, and solves after a
rebuild stay bitwise equal to the oracle.  Needs an MI355X: -m gpu.

D and CF (floats) must be bitwise equal.  CD holds double cosines of the cone and tangent
radii: the host evaluates them with glibc's cos (the reference's), the device with its own,
and the two differ in the last bit for ~1.6 % of inputs (tests/test_gpu_libm.py).  The solve
only compares CD entries with float-valued doubles (ik_open_cone_3d.cpp:285-321, :358-381), so
CD must be *observably* equal: the same bits, or adjacent doubles with no float between them."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", 0))


def _float_between(lo, hi):
    """Is there a float f with lo < f <= hi (elementwise, lo <= hi)?"""
    f = hi.astype(np.float32)
    f = np.where(f.astype(np.float64) > hi, np.nextafter(f, np.float32(-np.inf)), f)
    return f.astype(np.float64) > lo


def _assert_tables_equal(a, b, what):
    for name, x, y in zip(("D", "CF", "CD"), a, b):
        assert x.shape == y.shape, (what, name)
        bad = np.argwhere(x.view(np.uint32 if x.dtype == np.float32 else np.uint64)
                          != y.view(np.uint32 if y.dtype == np.float32 else np.uint64))
        if name == "CD" and bad.size:
            xs, ys = x[tuple(bad.T)], y[tuple(bad.T)]
            lo, hi = np.minimum(xs, ys), np.maximum(xs, ys)
            ulps = np.abs(xs.view(np.int64) - ys.view(np.int64))
            assert (ulps <= 1).all() and not _float_between(lo, hi).any() and \
                np.array_equal(lo.astype(np.float32), hi.astype(np.float32)), \
                f"{what} CD: {len(bad)} entries differ observably"
            continue
        assert bad.size == 0, f"{what} {name}: {len(bad)} entries differ, first {bad[:4].tolist()}"


def _topologies():
    parents = [-1, 0, 1, 2, -1, 4, 5, 6, 6]
    return [
        ("c2", W.topology(2)), ("c3", W.topology(3)), ("c4", W.topology(4)), ("c5", W.topology(5)),
        ("multi_root_3cones", W.custom_topology(parents, [0, 3, 7, 8], constrained=[1, 2, 5, 6, 7], cones_per_bone=3,
                                                 twist=(math.radians(-30), math.radians(90)), iterations=10)),
    ]


@pytest.mark.parametrize("name,topo", _topologies(), ids=lambda x: x if isinstance(x, str) else "")
def test_gpu_setup_equals_host_setup(mbik, name, topo):
    import torch
    n = 256 if topo.parents.shape[0] < 100 else 64
    wl = W.generate(2, n, first=123, topo=topo)
    plan = Plan.from_workload(wl)
    host = plan.setup_tables()
    pose, cones, twist = _dev(torch, wl.pose), _dev(torch, wl.cones), _dev(torch, wl.twist)
    plan.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    _assert_tables_equal(plan.setup_tables(), host, name)


def test_gpu_setup_random_radii(oracle, mbik):
    """Per-skeleton random cone radii and twist ranges (every cosine a different input):
    tables observably equal, and the solve after the GPU rebuild bitwise equal to the oracle."""
    import torch
    wl = W.generate(2, 128, first=31)
    rng = np.random.default_rng(7)
    wl.cones[..., 3] = rng.uniform(0.05, 1.2, wl.cones.shape[:-1]).astype(np.float32)
    wl.twist[..., 1] = rng.uniform(0.1, 6.0, wl.twist.shape[:-1]).astype(np.float32)
    plan = Plan.from_workload(wl)
    host = plan.setup_tables()
    pose, cones, twist = _dev(torch, wl.pose), _dev(torch, wl.cones), _dev(torch, wl.twist)
    plan.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    _assert_tables_equal(plan.setup_tables(), host, "random radii")
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, "solve after GPU setup, random radii")


def test_gpu_setup_from_new_poses_matches_a_fresh_plan(oracle, mbik):
    """Rebuild a plan's setup from other skeletons' setup poses/cones on the GPU: tables and
    solves equal a plan built on the host from those inputs."""
    import torch
    a = W.generate(5, 24, first=0)
    b = W.generate(5, 24, first=5000)
    plan = Plan.from_workload(a)
    pose, cones, twist = _dev(torch, b.pose), _dev(torch, b.cones), _dev(torch, b.twist)
    plan.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    fresh = Plan.from_workload(b)
    _assert_tables_equal(plan.setup_tables(), fresh.setup_tables(), "C5 rebuilt")
    ref = oracle.Oracle(b).solve(b.pose, b.targets, threads=8)
    assert_parity(plan.solve_host(b.pose, b.targets), ref, "C5 solve after GPU setup")


def test_gpu_setup_partial_range(mbik):
    import torch
    a = W.generate(2, 64, first=0)
    b = W.generate(2, 64, first=777)
    plan = Plan.from_workload(a)
    before = plan.setup_tables()
    pose, cones, twist = _dev(torch, b.pose[10:20]), _dev(torch, b.cones[10:20]), _dev(torch, b.twist[10:20])
    plan.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), first=10, count=10,
                       stream=torch.cuda.current_stream().cuda_stream)
    after = plan.setup_tables()
    fresh = Plan.from_workload(b).setup_tables()
    for x, y, z in zip(before, after, fresh):
        assert np.array_equal(x[..., :10], y[..., :10]) and np.array_equal(x[..., 20:], y[..., 20:])
    _assert_tables_equal([y[..., 10:20] for y in after], [z[..., 10:20] for z in fresh], "partial range")
