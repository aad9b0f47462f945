"""constraint_mode (ik_bone_segment_3d.cpp:142) on the GPU vs the oracle, bitwise, over several
frames: the reference's IKNode3D caches outlive a frame, so each case runs a sequence of
mbik_solve calls on one plan beside one oracle object graph."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_edge_cases import CASES
from .test_gpu_fuzz import random_case
from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def animate(pose, rng, angle=0.2):
    """Next frame's input: every bone's rotation turned by a small random rotation (an
    animation track); about a quarter of the bones keep their pose bitwise."""
    out = pose.copy()
    n, B = pose.shape[:2]
    axis = rng.normal(size=(n, B, 3))
    axis /= np.linalg.norm(axis, axis=-1, keepdims=True)
    a = rng.uniform(0, angle, (n, B, 1))
    dq = np.concatenate([axis * np.sin(a / 2), np.cos(a / 2)], -1)
    q = pose[..., 0:4].astype(np.float64)
    x1, y1, z1, w1 = dq[..., 0], dq[..., 1], dq[..., 2], dq[..., 3]
    x2, y2, z2, w2 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    prod = np.stack([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2], -1)
    keep = rng.random((n, B)) < 0.25
    out[..., 0:4] = np.where(keep[..., None], pose[..., 0:4], prod.astype(np.float32))
    return out


def run_frames(oracle, wl, frames=4, stab=0, seed=0, lanes=0, spw=0, roles=None, expect_roles=None):
    """Frame 1 starts from the setup pose; then the output is fed back (a still skeleton)
    and, every other frame, animated.  roles: mbik_plan_set_wave_roles (None: the default)."""
    rng = np.random.default_rng(seed)
    ref_o = oracle.Oracle(wl, constraint_mode=True, stabilization_passes=stab)
    plan = Plan.from_workload(wl, constraint_mode=True, stabilization_passes=stab, lanes=lanes)
    if roles is not None:
        plan.set_wave_roles(roles)
    if spw:
        plan.set_layout(lanes, spw, 0)
    pose = wl.pose.copy()
    changed = 0
    for f in range(frames):
        ref = ref_o.solve(pose, wl.targets, threads=4)
        got = plan.solve_host(pose, wl.targets)
        assert_parity(got, ref, f"frame {f}")
        changed += int((got[..., 0:4] != pose[..., 0:4]).any(-1).sum())
        pose = animate(ref, rng) if f % 2 else ref
    if expect_roles is not None:
        assert plan.info()["wave_roles"] == expect_roles
    plan.close()
    ref_o.close()
    return changed


@pytest.mark.parametrize("cfg,n", [(1, 4), (2, 96), (3, 40), (5, 6)])
def test_configs_over_frames(oracle, mbik, cfg, n):
    changed = run_frames(oracle, W.generate(cfg, n), frames=4, seed=cfg)
    if cfg in (2, 5):  # constrained configs: the snaps move bones
        assert changed > 0


@pytest.mark.parametrize("stab", [1, 2])
def test_with_stabilization(oracle, mbik, stab):
    run_frames(oracle, W.generate(2, 48), frames=3, stab=stab, seed=10 + stab)


@pytest.mark.parametrize("name", list(CASES))
def test_topology_edge_cases(oracle, mbik, name):
    parents, pins, cons, ncones, twist = CASES[name]
    topo = W.custom_topology(parents, pins, cons, cones_per_bone=ncones, twist=twist)
    run_frames(oracle, W.generate(11, 16, topo=topo), frames=3, seed=20)


@pytest.mark.parametrize("seed", range(16))
def test_random_configurations(oracle, mbik, seed):
    wl, stab, _ = random_case(seed)
    run_frames(oracle, wl, frames=3, stab=stab, seed=seed)


def test_tight_limits_many_snaps(oracle, mbik):
    """Narrow cones and twist: nearly every bone-step swings and twists, so stale caches
    (rotate_local_with_global without propagation) are hit constantly."""
    topo = W.custom_topology([-1, 0, 1, 2, 3, 1, 5, 6, 7], [4, 8], list(range(1, 9)), cones_per_bone=2,
                             twist=(math.radians(-3), math.radians(6)), iterations=6)
    wl = W.generate(15, 24, topo=topo)
    wl.cones[..., 3] = np.float32(math.radians(4))
    assert run_frames(oracle, wl, frames=4, seed=30) > 0, "no bone was snapped"


def test_layout_override_is_ignored(oracle, mbik):
    run_frames(oracle, W.generate(2, 24), frames=2, lanes=8, seed=40)


def test_rebuild_setup_restarts_the_node_tree(oracle, mbik, torch_dev):
    """mbik_plan_rebuild_setup == _bone_list_changed: fresh node caches from the new setup."""
    torch, dev = torch_dev
    wl = W.generate(2, 32)
    plan = Plan.from_workload(wl, constraint_mode=True)
    pose = wl.pose
    for _ in range(2):                      # advance the caches
        pose = plan.solve_host(pose, wl.targets)
    sp = torch.from_numpy(wl.pose).to(dev)
    cones = torch.from_numpy(np.ascontiguousarray(wl.cones)).to(dev)
    twist = torch.from_numpy(np.ascontiguousarray(wl.twist)).to(dev)
    plan.rebuild_setup(sp.data_ptr(), cones.data_ptr(), twist.data_ptr())
    torch.cuda.synchronize()
    fresh = oracle.Oracle(wl, constraint_mode=True)
    assert_parity(plan.solve_host(wl.pose, wl.targets), fresh.solve(wl.pose, wl.targets), "after rebuild")
    plan.close()


def test_segment_solve(oracle, mbik, torch_dev):
    """mbik_segment_solve in constraint_mode == IKBoneSegment3D::segment_solver."""
    torch, dev = torch_dev
    wl = W.generate(2, 16)
    ref_o = oracle.Oracle(wl, constraint_mode=True)
    plan = Plan.from_workload(wl, constraint_mode=True)
    pose = wl.pose.copy()
    for seg in range(ref_o.segment_count()):
        ref = ref_o.segment_solve(seg, pose, wl.targets)
        d = torch.from_numpy(pose).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, d.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(d.cpu().numpy(), ref, f"segment {seg}")
        pose = ref
    plan.close()


def test_autotune_keeps_the_node_caches(oracle, mbik, torch_dev):
    """mbik_plan_autotune in constraint_mode times lane counts from a saved copy of the node
    caches and restores it: the frames around it match the oracle's uninterrupted sequence."""
    torch, dev = torch_dev
    wl = W.generate(5, 8)
    ref_o = oracle.Oracle(wl, constraint_mode=True)
    plan = Plan.from_workload(wl, constraint_mode=True)
    pose = wl.pose.copy()
    for f in range(3):
        if f == 1:
            pi = torch.from_numpy(pose).to(dev)
            tg = torch.from_numpy(wl.targets).to(dev)
            po = torch.empty_like(pi)
            plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
            torch.cuda.synchronize()
        ref = ref_o.solve(pose, wl.targets)
        got = plan.solve_host(pose, wl.targets)
        assert_parity(got, ref, f"frame {f}")
        pose = ref
    plan.close()


@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 16])
def test_lane_counts(oracle, mbik, lanes):
    run_frames(oracle, W.generate(5, 6), frames=2, lanes=lanes, seed=60)


@pytest.mark.parametrize("cfg,n,lanes,spw,stab", [(2, 3200, 4, 3, 0), (5, 2048, 4, 2, 0), (5, 1024, 2, 1, 2), (2, 700, 1, 64, 0)])
def test_multiwave_blocks_and_partial_waves(oracle, mbik, cfg, n, lanes, spw, stab):
    """constraint_mode blocks of several waves sharing one LDS copy of the topology, each wave
    holding fewer skeletons than 64 / K (cmode_shape: enough blocks for every CU, then as many
    waves per block as fit): the same bits over animated frames."""
    wl = W.generate(cfg, n, first=123)
    run_frames(oracle, wl, frames=3, stab=stab, seed=70 + cfg, lanes=lanes, spw=spw)
