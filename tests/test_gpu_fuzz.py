"""Randomized topologies and configurations (seeded, reproducible): random forests with
shuffled bone order and several roots, random pins / constraints / cone counts / twist
ranges / pin weights, priorities and propagation, damping, iteration counts, stabilization
and lane counts -- every case bitwise equal to the oracle.  Needs an MI355X: -m gpu."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu
N_CASES = 48


def random_case(seed: int, rest: str = "plus_y"):
    rng = np.random.default_rng(1000 + seed)
    B = int(rng.integers(2, 40))
    n_roots = 1 if rng.random() < 0.7 else int(rng.integers(2, 4))
    parents = [-1] * B
    for b in range(n_roots, B):
        # mostly chains with occasional branching
        parents[b] = b - 1 if rng.random() < 0.6 else int(rng.integers(0, b))
    perm = rng.permutation(B)                 # shuffle the bone order (parents need not come first)
    inv = np.empty(B, int)
    inv[perm] = np.arange(B)
    parents = [(-1 if parents[perm[i]] < 0 else int(inv[parents[perm[i]]])) for i in range(B)]
    n_pins = int(rng.integers(1, min(8, B) + 1))
    pins = sorted(rng.choice(B, n_pins, replace=False).tolist())
    with_parent = [b for b in range(B) if parents[b] >= 0]
    n_cons = int(rng.integers(0, len(with_parent) + 1)) if with_parent else 0
    constrained = sorted(rng.choice(with_parent, n_cons, replace=False).tolist()) if n_cons else []
    cones_per_bone = int(rng.integers(0, 4))
    twist = (float(rng.uniform(-math.pi, math.pi)), float(rng.uniform(0.05, 2 * math.pi)))
    topo = W.custom_topology(parents, pins, constrained, cones_per_bone=cones_per_bone, twist=twist,
                             iterations=int(rng.integers(1, 13)), name=f"fuzz{seed}")
    wl = W.generate(9, 6, first=seed * 7, topo=topo, rest=rest)
    P, C = len(pins), len(constrained)
    wl.pin_weight = rng.choice([0.0, 0.3, 1.0, 2.5], P).astype(np.float32)
    wl.pin_weight[int(rng.integers(0, P))] = 1.0          # at least one weighted pin
    wl.pin_priority = rng.choice([0.0, 0.2, 0.5, 1.0], (P, 3)).astype(np.float32)
    wl.pin_propagation = rng.choice([0.0, 0.5, 1.0], P).astype(np.float32)
    if C:
        wl.cone_count = rng.integers(0, cones_per_bone + 1, C).astype(np.int32)
    wl.default_damp = float(rng.choice([math.radians(2.0), math.radians(5.0), math.radians(30.0)]))
    if rng.random() < 0.3:
        wl.bone_damp = rng.uniform(0.01, 0.5, int(rng.integers(1, B + 1))).astype(np.float32)
    stab = int(rng.choice([0, 0, 1, 2]))
    lanes = int(rng.choice([0, 1, 4]))
    return wl, stab, lanes


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_configuration_bitwise(oracle, mbik, seed):
    wl, stab, lanes = random_case(seed)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=4)
    plan = Plan.from_workload(wl, lanes=lanes, stabilization_passes=stab)
    got = plan.solve_host(wl.pose, wl.targets)
    assert_parity(got, ref, f"fuzz seed {seed} (B={wl.bone_count}, stab={stab}, lanes={lanes})")


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_configuration_random_layout_bitwise(oracle, mbik, seed):
    """The same random rigs on a random launch layout: heading staging, state placement
    (LDS / locals / all in device memory), waves per SIMD, checkpoint interval and skeletons
    per block -- still bitwise equal to the oracle."""
    wl, stab, lanes = random_case(seed)
    rng = np.random.default_rng(5000 + seed)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=4)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    staging, placement, waves = int(rng.integers(0, 2)), int(rng.integers(0, 3)), int(rng.integers(1, 3))
    interval, spw = int(rng.choice([0, 1, 2, 3, 1 << 20])), int(rng.choice([0, 1, 3, 5]))
    plan.set_layout(lanes, spw, interval)
    plan.set_heading_staging(staging)
    plan.set_locals_placement(placement)
    plan.set_waves_per_simd(waves)
    got = plan.solve_host(wl.pose, wl.targets)
    assert_parity(got, ref, f"fuzz seed {seed} layout staging={staging} placement={placement} waves={waves} "
                            f"interval={interval} spw={spw} lanes={lanes} stab={stab}")
