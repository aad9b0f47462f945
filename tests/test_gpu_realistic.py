"""Realistic rest poses on the GPU vs the oracle, bitwise.  Needs an
MI355X: -m gpu.

``workloads.generate(rest="realistic")`` puts child offsets in random directions (tilted up
to 110 degrees off +Y, so multi-child bones' children point different ways), rolls every bone
about its own +Y and gives it a non-uniform scale; ``"realistic_unit_scale"`` keeps scale 1
(the long constrained C5 rig overflows in the reference's own arithmetic with any non-unit
scale).  On these rigs:
  * update_default_bone_direction_transform (ik_bone_3d.cpp:57-93) takes the general
    ``Quaternion(child_centroid, bone_Y)`` branch, so the bone-direction frames D are not the
    identity -- asserted below, so the branch is proven to run;
  * the tip-heading basis columns (ik_effector_3d.cpp:118-149) and the swing's bone heading
    (ik_kusudama_3d.cpp:347-376) see those frames;
  * get_rotation_quaternion's orthonormalization and get_scale (ik_bone_3d.cpp:161-179) see
    non-unit, non-uniform scales.
Every kernel variant is compared: the default launch, the helper wave, placement 2 with
split-exchange headings, constraint_mode over frames, segment_solve, GPU-built setup tables
and device-built plans, and the randomized rigs of test_gpu_fuzz."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, plans_from_device

from .test_gpu_constraint_mode import run_frames
from .test_gpu_fuzz import random_case
from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)
from .test_gpu_setup import _assert_tables_equal, _dev

pytestmark = pytest.mark.gpu

REST = {1: "realistic", 2: "realistic", 3: "realistic", 4: "realistic", 5: "realistic_unit_scale"}
IDENTITY9 = np.eye(3, dtype=np.float32).reshape(9)


def realistic(cfg, n, first=0, rest=None):
    return W.generate(cfg, n, first=first, rest=rest or REST[cfg])


def _d_not_identity(plan):
    D, _, _ = plan.setup_tables()                       # [bone][9][n]
    off = np.abs(D - IDENTITY9[None, :, None]).max(axis=1)
    return int((off > 1e-3).sum()), off.size


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_bone_direction_frames_take_the_general_branch(mbik, cfg):
    """The realistic rigs' D rows are rotations away from the identity for most bones with
    children; the +Y rigs' are all (numerically) the identity -- the branch the round-3 suite
    never left."""
    plan = Plan.from_workload(realistic(cfg, 16))
    moved, total = _d_not_identity(plan)
    assert moved > total // 2, f"C{cfg}: only {moved}/{total} bone-direction frames left the identity"
    plain = Plan.from_workload(W.generate(cfg, 16))
    assert _d_not_identity(plain)[0] == 0


@pytest.mark.parametrize("cfg,n", [(1, 4), (2, 96), (3, 96), (4, 24), (5, 6)])
@pytest.mark.parametrize("lanes", [0, 1, 4])
def test_realistic_configs_bitwise(oracle, mbik, cfg, n, lanes):
    wl = realistic(cfg, n, first=3000)
    assert not np.allclose(wl.pose[..., 7:10], 1.0) or cfg == 5
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, lanes=lanes)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"realistic C{cfg} lanes={lanes}")


@pytest.mark.parametrize("cfg,n", [(1, 8), (2, 48), (4, 16), (5, 6)])
def test_realistic_helper_wave(oracle, mbik, cfg, n):
    wl = realistic(cfg, n, first=3100)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_helper_wave(1)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"realistic C{cfg} helper wave")


@pytest.mark.parametrize("cfg,n,layout", [
    (4, 40, (4, 16, 1, 4, 2, 2)), (4, 40, (4, 16, 2, 5, 2, 2)), (5, 12, (8, 8, 1, 4, 2, 2)),
    (5, 12, (8, 8, 2, 5, 2, 1)), (2, 70, (4, 16, 1, 4, 2, 2)), (3, 70, (4, 16, 4, 4, 1, 2))])
def test_realistic_state_in_device_memory_split_exchange(oracle, mbik, cfg, n, layout):
    """Placement 2 (whole state in device memory, skeleton-tiled tables) with split-exchange
    heading staging (4/5) and two waves per SIMD: the layouts autotune picks for C3-C5."""
    lanes, spw, interval, staging, placement, waves = layout
    wl = realistic(cfg, n, first=3200)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(lanes, spw, interval)
    plan.set_heading_staging(staging)
    plan.set_locals_placement(placement)
    plan.set_waves_per_simd(waves)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["state_placement"] == placement
    assert_parity(got, ref, f"realistic C{cfg} layout {layout}")


@pytest.mark.parametrize("cfg,n", [(2, 48), (3, 24), (5, 4)])
def test_realistic_constraint_mode_over_frames(oracle, mbik, cfg, n):
    changed = run_frames(oracle, realistic(cfg, n, first=3300), frames=4, seed=70 + cfg)
    if cfg in (2, 5):
        assert changed > 0


@pytest.mark.parametrize("stab", [1, 2])
def test_realistic_stabilization(oracle, mbik, stab):
    wl = realistic(2, 32, first=3400)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"realistic C2 stabilization {stab}")


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_realistic_segment_solve(oracle, mbik, torch_dev, cfg):
    torch, dev = torch_dev
    wl = realistic(cfg, 8, first=3500)
    o = oracle.Oracle(wl)
    plan = Plan.from_workload(wl)
    nseg = plan.info()["segment_count"]
    for seg in sorted({0, nseg // 2, nseg - 1}):
        ref = o.segment_solve(seg, wl.pose, wl.targets)
        pose = torch.from_numpy(wl.pose.copy()).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, pose.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(pose.cpu().numpy(), ref, f"realistic C{cfg} segment {seg}")


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_realistic_gpu_setup_equals_host_setup(oracle, mbik, cfg):
    """mbik_plan_rebuild_setup derives D / CF / CD on the device (setup.h): equal to the host
    builder's on the general arc branch too, and the solve after it bitwise."""
    import torch
    wl = realistic(cfg, 64, first=3600)
    plan = Plan.from_workload(wl)
    host = plan.setup_tables()
    pose, cones, twist = _dev(torch, wl.pose), _dev(torch, wl.cones), _dev(torch, wl.twist)
    plan.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    _assert_tables_equal(plan.setup_tables(), host, f"realistic C{cfg}")
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"realistic C{cfg} after GPU setup")


def test_realistic_device_built_plans(oracle, mbik):
    """mbik_plan_create_device: topology and setup built on the GPU for a crowd of distinct
    realistic rigs, each solve bitwise equal to the oracle."""
    import torch
    wls = [realistic(2, 32, first=3700), realistic(4, 16, first=3700), realistic(5, 4, first=3700)]
    rigs = [(wl.topo.parents, wl.pins(), wl.constraints(),
             dict(iterations=wl.topo.iterations, default_damp=wl.default_damp, max_cones=wl.cones.shape[2]))
            for wl in wls]
    keep = [(_dev(torch, wl.pose), _dev(torch, wl.cones), _dev(torch, wl.twist)) for wl in wls]
    plans = plans_from_device(rigs, [wl.n for wl in wls], [k[0].data_ptr() for k in keep],
                              [k[1].data_ptr() if wl.topo.constrained.size else 0 for k, wl in zip(keep, wls)],
                              [k[2].data_ptr() if wl.topo.constrained.size else 0 for k, wl in zip(keep, wls)])
    for wl, plan in zip(wls, plans):
        ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
        assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"device-built realistic {wl.topo.name}")


@pytest.mark.parametrize("seed", range(24))
def test_realistic_random_configuration_bitwise(oracle, mbik, seed):
    """test_gpu_fuzz's random forests, pins, constraints and settings on realistic rest poses
    (non-unit scale on even seeds): bitwise, on the default and on a random launch layout."""
    wl, stab, lanes = random_case(seed, rest="realistic" if seed % 2 == 0 else "realistic_unit_scale")
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=4)
    fin = np.isfinite(ref).all(axis=(1, 2))
    plan = Plan.from_workload(wl, lanes=lanes, stabilization_passes=stab)
    got = plan.solve_host(wl.pose, wl.targets)
    _assert_same_bits_or_both_nonfinite(got, ref, fin, f"realistic fuzz seed {seed}")
    rng = np.random.default_rng(9000 + seed)
    plan.set_heading_staging(int(rng.integers(0, 2)))
    plan.set_locals_placement(int(rng.integers(0, 3)))
    plan.set_waves_per_simd(int(rng.integers(1, 3)))
    got = plan.solve_host(wl.pose, wl.targets)
    _assert_same_bits_or_both_nonfinite(got, ref, fin, f"realistic fuzz seed {seed}, random layout")


def _assert_same_bits_or_both_nonfinite(got, ref, fin, what):
    """Finite skeletons bitwise; a skeleton whose oracle solve overflowed must overflow on the
    GPU at the same values (NaN payloads aside)."""
    if fin.any():
        assert_parity(got[fin], ref[fin], what)
    if (~fin).any():
        g, r = got[~fin], ref[~fin]
        assert np.array_equal(np.isnan(g), np.isnan(r)), f"{what}: NaN placement differs"
        ok = ~np.isnan(r)
        assert np.array_equal(g[ok].view(np.uint32), r[ok].view(np.uint32)), f"{what}: non-NaN values differ"


def test_realistic_scaled_c5_overflows_like_the_reference(oracle, mbik):
    """Non-unit scale on the constrained C5 rig overflows in the reference's own arithmetic
    within two iterations; the GPU overflows identically (same NaN placement, same finite
    values, same per-skeleton non-finite flags through mbik_solve_checked)."""
    import torch
    wl = W.generate(5, 4, first=3800, rest="realistic")
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=4)
    fin = np.isfinite(ref).all(axis=(1, 2))
    assert not fin.all()
    plan = Plan.from_workload(wl)
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    nf = torch.zeros(wl.n, dtype=torch.uint8, device=dev)
    plan.solve_checked(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), nf.data_ptr())
    torch.cuda.synchronize()
    _assert_same_bits_or_both_nonfinite(po.cpu().numpy(), ref, fin, "scaled C5")
    flags = nf.cpu().numpy()
    assert not flags[fin].any() and flags[~fin].all(), flags


def test_realistic_scale_reaches_the_output(oracle, mbik):
    """get_scale (ik_bone_3d.cpp:178) on non-uniform locals: the output scale column is not 1
    and matches the oracle bit for bit (the parity tests above include it; this pins that the
    case is actually exercised)."""
    wl = realistic(2, 16, first=3900)
    got = Plan.from_workload(wl).solve_host(wl.pose, wl.targets)
    assert np.abs(got[..., 7:10] - 1).max() > 0.1
    assert (np.abs(got[..., 7] - got[..., 8]) > 1e-3).any(), "no non-uniform scale in the output"
    assert_parity(got, oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8), "realistic scale output")

