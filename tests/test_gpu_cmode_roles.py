"""constraint_mode with wave roles (cmode.h mbik_cmode_kernel_rw): the K roles of the sibling
schedule as the block's waves, a lane per skeleton, and a multi-effector segment's effector reads
split over its group of waves (plan.cpp cm_split_groups) -- bitwise against the oracle's
persistent object graph over animated frames, as test_gpu_constraint_mode does for the classic
kernel."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_constraint_mode import animate, run_frames
from .test_gpu_edge_cases import CASES
from .test_gpu_fuzz import random_case
from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lanes", [2, 4, 8])
@pytest.mark.parametrize("cfg,n", [(1, 4), (2, 96), (3, 40), (4, 24), (5, 70)])
def test_configs_over_frames(oracle, mbik, cfg, n, lanes):
    run_frames(oracle, W.generate(cfg, n, first=7), frames=4, seed=cfg, lanes=lanes, roles=1, expect_roles=1)


@pytest.mark.parametrize("lanes,spw", [(4, 16), (8, 32), (2, 7), (8, 64), (4, 1)])
def test_skeletons_per_block(oracle, mbik, lanes, spw):
    """Partly filled blocks (spw < 64) and a launch that is not a multiple of the block."""
    run_frames(oracle, W.generate(5, 150, first=3), frames=3, seed=80 + spw, lanes=lanes, spw=spw, roles=1, expect_roles=1)


@pytest.mark.parametrize("name", list(CASES))
def test_topology_edge_cases(oracle, mbik, name):
    parents, pins, cons, ncones, twist = CASES[name]
    topo = W.custom_topology(parents, pins, cons, cones_per_bone=ncones, twist=twist)
    run_frames(oracle, W.generate(11, 16, topo=topo), frames=3, seed=20, lanes=4, roles=1)


@pytest.mark.parametrize("seed", range(16))
def test_random_configurations(oracle, mbik, seed):
    """test_gpu_fuzz's random forests (stabilized ones run the classic kernel: no wave roles)."""
    wl, stab, _ = random_case(seed)
    run_frames(oracle, wl, frames=3, stab=stab, seed=seed, lanes=8, roles=1, expect_roles=0 if stab else None)


def test_tight_limits_many_snaps(oracle, mbik):
    topo = W.custom_topology([-1, 0, 1, 2, 3, 1, 5, 6, 7], [4, 8], list(range(1, 9)), cones_per_bone=2,
                             twist=(math.radians(-3), math.radians(6)), iterations=6)
    wl = W.generate(15, 24, topo=topo)
    wl.cones[..., 3] = np.float32(math.radians(4))
    assert run_frames(oracle, wl, frames=4, seed=30, lanes=2, roles=1, expect_roles=1) > 0


def test_shared_chains_stay_on_one_wave(oracle, mbik):
    """A root segment whose effectors pair up below it (two limbs of two fingers each, and a
    third limb's tip): the fingers of one limb share that limb's dirty chain below the trunk (the
    root bone), so they are one cluster, read in order by one wave (plan.cpp cm_split_groups)."""
    parents = [-1, 0, 1, 2, 3, 3, 0, 6, 7, 8, 8, 0, 11, 12]
    #          root, limb A 1-3, fingers 4 5; limb B 6-8, fingers 9 10; limb C 11-13 (tip 13)
    topo = W.custom_topology(parents, [13, 4, 5, 9, 10], list(range(1, 14)), cones_per_bone=1,
                             twist=(math.radians(-20), math.radians(40)), iterations=8)
    run_frames(oracle, W.generate(16, 40, topo=topo), frames=4, seed=31, lanes=8, roles=1, expect_roles=1)


def test_segment_solve(oracle, mbik, torch_dev):
    torch, dev = torch_dev
    wl = W.generate(5, 20)
    ref_o = oracle.Oracle(wl, constraint_mode=True)
    plan = Plan.from_workload(wl, constraint_mode=True, lanes=8)
    plan.set_wave_roles(1)
    pose = wl.pose.copy()
    for seg in range(ref_o.segment_count()):
        ref = ref_o.segment_solve(seg, pose, wl.targets)
        d = torch.from_numpy(pose).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, d.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(d.cpu().numpy(), ref, f"segment {seg}")
        pose = ref
    assert plan.info()["wave_roles"] == 1
    plan.close()


def test_autotune_times_wave_roles_and_keeps_the_caches(oracle, mbik, torch_dev):
    """mbik_plan_autotune now also times wave-roles layouts: the frames around it still match the
    oracle's uninterrupted sequence, whichever layout it keeps."""
    torch, dev = torch_dev
    wl = W.generate(5, 300)
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
        ref = ref_o.solve(pose, wl.targets, threads=4)
        got = plan.solve_host(pose, wl.targets)
        assert_parity(got, ref, f"frame {f}")
        pose = ref
    plan.close()


def test_save_load_keeps_wave_roles(oracle, mbik):
    wl = W.generate(2, 64)
    ref_o = oracle.Oracle(wl, constraint_mode=True)
    plan = Plan.from_workload(wl, constraint_mode=True, lanes=4)
    plan.set_wave_roles(1)
    pose = plan.solve_host(wl.pose, wl.targets)
    assert_parity(pose, ref_o.solve(wl.pose, wl.targets), "frame 0")
    blob = plan.save()
    plan.close()
    plan2 = Plan.load(blob)
    got = plan2.solve_host(pose, wl.targets)
    assert_parity(got, ref_o.solve(pose, wl.targets), "frame 1 after load")
    assert plan2.info()["wave_roles"] == 1
    plan2.close()


def test_c5_full_size_two_frames(oracle, mbik):
    """The constraint_mode bench line's layout at its timed size: C5, 16,384
    skeletons on the wave-roles kernel with K = 8 waves and 64 skeletons per block, two frames (the
    second from the first's output, animated).  The node caches of every skeleton advance on the
    GPU; oracle object graphs of the skeletons at the start, the middle and the end of the batch
    take the same inputs and must give the same bits each frame."""
    n = 16384
    wl = W.generate(5, n)
    plan = Plan.from_workload(wl, constraint_mode=True, lanes=8)
    plan.set_wave_roles(1)
    windows = [(0, 3), (n // 2 - 1, 3), (n - 4, 4)]
    graphs = [oracle.Oracle(W.generate(5, k, first=f), constraint_mode=True) for f, k in windows]
    rng = np.random.default_rng(91)
    pose = wl.pose
    for frame in range(2):
        got = plan.solve_host(pose, wl.targets)
        info = plan.info()
        assert info["wave_roles"] == 1 and info["lanes_per_skeleton"] == 8 and info["skeletons_per_block"] == 64, info
        assert np.isfinite(got).all()
        for (f, k), o in zip(windows, graphs):
            ref = o.solve(np.ascontiguousarray(pose[f:f + k]), np.ascontiguousarray(wl.targets[f:f + k]), threads=4)
            assert_parity(got[f:f + k], ref, f"C5 constraint_mode K8 frame {frame} @{f}")
        pose = animate(got, rng)
    plan.close()
    for o in graphs:
        o.close()
