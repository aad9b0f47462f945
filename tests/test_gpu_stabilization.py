"""Stabilization passes (IKBoneSegment3D::_set_optimal_rotation retry loop,
ik_bone_segment_3d.cpp:114-127,163-180; root segments only) on the HIP path vs the
oracle, bitwise.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n", [(1, 8), (2, 64), (3, 64), (4, 16), (5, 4)])
@pytest.mark.parametrize("passes", [1, 3])
@pytest.mark.parametrize("lanes", [0, 1])
def test_stabilization_bitwise_vs_oracle(oracle, mbik, cfg, n, passes, lanes):
    wl = W.generate(cfg, n, first=2000)
    ref = oracle.Oracle(wl, stabilization_passes=passes).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, lanes=lanes, stabilization_passes=passes)
    got = plan.solve_host(wl.pose, wl.targets)
    assert_parity(got, ref, f"C{cfg} passes={passes} lanes={lanes}")


def _spine_topology():
    """A 4-bone root segment (spine) under two 5-bone limbs: multi-bone root segments are
    where stabilization can reject (a single-bone root always accepts, previous_deviation
    being reset to infinity after the segment root)."""
    parents = [-1, 0, 1, 2]
    tips = []
    for _ in range(2):
        p = 3
        for _ in range(5):
            parents.append(p)
            p = len(parents) - 1
        tips.append(p)
    return W.custom_topology(parents, tips, np.arange(1, len(parents)), cones_per_bone=2, twist=(0.0, 1.0),
                             iterations=6)


@pytest.mark.parametrize("passes", [1, 2, 5])
@pytest.mark.parametrize("lanes", [0, 1, 4])
def test_stabilization_spine_root(oracle, mbik, passes, lanes):
    wl = W.generate(2, 48, topo=_spine_topology())
    base = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    ref = oracle.Oracle(wl, stabilization_passes=passes).solve(wl.pose, wl.targets, threads=8)
    assert not np.array_equal(base, ref)  # the retry path changes this solve
    got = Plan.from_workload(wl, lanes=lanes, stabilization_passes=passes).solve_host(wl.pose, wl.targets)
    assert_parity(got, ref, f"spine passes={passes} lanes={lanes}")


def test_stabilization_multi_root_and_pinned_root(oracle, mbik):
    """Two root segments (both stabilized) and a pinned root bone."""
    parents = [-1, 0, 1, 2, -1, 4, 5, 6, 6]
    topo = W.custom_topology(parents, [0, 3, 7, 8], constrained=[1, 2, 5, 6], cones_per_bone=2, twist=(0.0, 1.0),
                             iterations=12)
    wl = W.generate(2, 32, topo=topo)
    for passes in (1, 4):
        ref = oracle.Oracle(wl, stabilization_passes=passes).solve(wl.pose, wl.targets, threads=8)
        got = Plan.from_workload(wl, stabilization_passes=passes).solve_host(wl.pose, wl.targets)
        assert_parity(got, ref, f"multi-root passes={passes}")
