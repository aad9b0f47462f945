"""Effector path sharing (HostPlan::seg_eff_lcp): consecutive effectors of a
segment start their walk from the previous effector's product at their branch point.  Random
branching rigs -- limbs with several fingers each, pins on the fingers and in the middle of
other pins' paths (an effector path that is a prefix of the next one's), constrained bones,
stale bone-direction caches after swings -- solved unstaged (the path that shares) in every
state placement and wave count, bitwise against the oracle."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def branching_rig(seed):
    rng = np.random.default_rng(seed)
    parents = [-1]
    pins = []

    def chain(parent, n):
        for _ in range(n):
            parents.append(parent)
            parent = len(parents) - 1
        return parent

    for _ in range(int(rng.integers(2, 4))):                      # limbs off the root
        limb = chain(0, int(rng.integers(2, 6)))
        if rng.random() < 0.5:
            pins.append(limb)                                      # a pin whose path prefixes its fingers'
        for _ in range(int(rng.integers(2, 5))):                   # fingers off the limb's end
            pins.append(chain(limb, int(rng.integers(1, 5))))
    order = rng.permutation(len(pins)) if rng.random() < 0.3 else np.arange(len(pins))
    pins = [pins[i] for i in order]                                # sometimes not in tree order
    B = len(parents)
    cons = sorted(int(b) for b in rng.choice(np.arange(1, B), size=int(rng.integers(0, B)), replace=False))
    return W.custom_topology(parents, pins, cons, cones_per_bone=int(rng.integers(1, 3)) if cons else 0,
                             twist=(-0.4, 1.2) if cons else None)


@pytest.mark.parametrize("seed", range(6))
def test_shared_path_walks_bitwise(oracle, mbik, seed):
    topo = branching_rig(1000 + seed)
    wl = W.generate(11, 24, first=seed * 100, topo=topo)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    for placement in (0, 2):
        for waves in (1, 2):
            plan = Plan.from_workload(wl)
            plan.set_heading_staging(0)
            plan.set_locals_placement(placement)
            plan.set_waves_per_simd(waves)
            assert_parity(plan.solve_host(wl.pose, wl.targets), ref,
                          f"rig {seed} placement {placement} waves {waves}")
            plan.close()
