"""Wave roles (mbik_plan_set_wave_roles, ABI 8): the north star's "one wavefront per segment".
A lane of a wave is one skeleton (64 per block) and the K roles of the sibling-segment schedule
are the block's K waves, meeting at a barrier per tree level (ik_bone_segment_3d.cpp:210-240's
post-order recursion); the whole state is in device memory.  Every such layout must be bitwise
equal to the oracle: C2-C5, +Y and realistic rest poses, both heading-slot kernel families, K =
2 / 4 / 8 waves at one and two waves per SIMD, checkpoint intervals, partial blocks,
segment_solve, solve_checked's non-finite flags, save/load and a fused group.  Needs an
MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_heading_slots import PRIORITIES, workload
from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)
from .test_gpu_realistic import realistic

pytestmark = pytest.mark.gpu

# (K waves per block, waves per SIMD): every built instantiation
ROLES = [(2, 1), (2, 2), (4, 1), (4, 2), (8, 2)]


def rw_plan(wl, k, wps, interval=0, **kw):
    plan = Plan.from_workload(wl, **kw)
    plan.set_layout(k, 0, interval)
    plan.set_waves_per_simd(wps)
    plan.set_wave_roles(1)
    return plan


def check_info(plan, k, wps):
    info = plan.info()
    assert info["wave_roles"] == 1, info
    assert info["lanes_per_skeleton"] == k and info["skeletons_per_block"] == 64
    assert info["state_placement"] == 2 and info["waves_per_simd"] == wps


@pytest.mark.parametrize("cfg,n", [(2, 70), (3, 130), (4, 70), (5, 66)])
@pytest.mark.parametrize("k,wps", ROLES)
def test_wave_roles_bitwise_vs_oracle(oracle, mbik, cfg, n, k, wps):
    """n = a full block plus a partial one: lanes past the batch must idle at every barrier."""
    wl = W.generate(cfg, n, first=51000 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = rw_plan(wl, k, wps)
    got = plan.solve_host(wl.pose, wl.targets)
    check_info(plan, k, wps)
    assert_parity(got, ref, f"C{cfg} wave roles K={k} wps={wps}")


@pytest.mark.parametrize("cfg,n", [(2, 40), (4, 40), (5, 20)])
@pytest.mark.parametrize("interval", [2, 3, 1 << 20])
def test_wave_roles_checkpoint_intervals(oracle, mbik, cfg, n, interval):
    wl = W.generate(cfg, n, first=52000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = rw_plan(wl, 4, 2, interval)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} wave roles interval={interval}")
    assert plan.info()["checkpoint_interval"] == interval


@pytest.mark.parametrize("cfg,n", [(2, 72), (3, 72), (4, 40), (5, 12)])
@pytest.mark.parametrize("k,wps", [(2, 1), (4, 2), (8, 2)])
def test_wave_roles_realistic_rest_poses(oracle, mbik, cfg, n, k, wps):
    wl = realistic(cfg, n, first=53000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = rw_plan(wl, k, wps)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} realistic wave roles K={k}")


@pytest.mark.parametrize("name", list(PRIORITIES))
@pytest.mark.parametrize("cfg,n", [(4, 24), (5, 8)])
def test_wave_roles_heading_slot_families(oracle, mbik, name, cfg, n):
    wl = workload(cfg, n, PRIORITIES[name], 54000 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = rw_plan(wl, 4, 2)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["heading_slots"] == (0x67 if name == "default" else 0)
    assert_parity(got, ref, f"C{cfg} {name} wave roles")


def test_wave_roles_fuzz_rigs(oracle, mbik):
    """Randomized rigs (multi-root, unsorted parents, pins mid-chain, 0-3 cones, twist): the
    schedule's rows and packed levels over the waves, whatever their shape."""
    from .test_gpu_fuzz import random_case
    for seed in range(12):
        wl, _, _ = random_case(seed)          # (stabilization excluded: wave roles refuse it)
        ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
        for k, wps in [(2, 1), (4, 2)]:
            plan = rw_plan(wl, k, wps)
            got = plan.solve_host(wl.pose, wl.targets)
            assert_parity(got, ref, f"fuzz seed {seed} wave roles K={k}")


def test_single_segment_rig_runs_without_wave_roles(oracle, mbik):
    """One role (C1: a single chain) is the classic 64-skeletons-per-wave layout; the plan
    reports wave_roles 0 and still solves exactly."""
    wl = W.generate(1, 9, first=3)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_wave_roles(1)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["wave_roles"] == 0
    assert_parity(got, ref, "C1 wave roles requested")


def test_wave_roles_refused_with_stabilization(oracle, mbik):
    wl = W.generate(2, 16, first=5)
    ref = oracle.Oracle(wl, stabilization_passes=2).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=2)
    plan.set_wave_roles(1)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["wave_roles"] == 0
    assert_parity(got, ref, "C2 stabilization, wave roles requested")


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_wave_roles_segment_solve(oracle, mbik, torch_dev, cfg):
    """mbik_segment_solve (IKBoneSegment3D::segment_solver) of single segments on a wave-roles
    plan equals the oracle's segment_solver."""
    torch, dev = torch_dev
    wl = W.generate(cfg, 70, first=55000)
    o = oracle.Oracle(wl)
    plan = rw_plan(wl, 4, 2)
    nseg = plan.info()["segment_count"]
    for seg in sorted({0, nseg // 2, nseg - 1}):
        ref = o.segment_solve(seg, wl.pose, wl.targets)
        pose = torch.from_numpy(wl.pose.copy()).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, pose.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(pose.cpu().numpy(), ref, f"C{cfg} wave roles segment {seg}")


def test_wave_roles_nonfinite_flags(oracle, mbik, torch_dev):
    """C5 with non-unit scales overflows in the reference's own arithmetic: the
    same bits as the classic launch, and the same per-skeleton flags -- an OR over the bones
    that every wave of the block wrote."""
    torch, dev = torch_dev
    wl = realistic(5, 70, first=56000, rest="realistic")
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    outs, flags = [], []
    for roles in (0, 1):
        plan = rw_plan(wl, 8, 2) if roles else Plan.from_workload(wl)
        po = torch.empty_like(pi)
        f = torch.full((wl.n,), 7, dtype=torch.uint8, device=dev)
        plan.solve_checked(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), f.data_ptr())
        torch.cuda.synchronize()
        outs.append(po.cpu().numpy())
        flags.append(f.cpu().numpy())
    # (NaN payloads may differ between builds; test_gpu_realistic compares NaN placement too)
    nan0, nan1 = np.isnan(outs[0]), np.isnan(outs[1])
    assert np.array_equal(nan0, nan1)
    assert np.array_equal(outs[0][~nan0].view(np.uint32), outs[1][~nan1].view(np.uint32))
    assert np.array_equal(flags[0], flags[1]) and set(np.unique(flags[1])) <= {0, 1}
    assert flags[1].sum() > 0


def test_wave_roles_save_load(oracle, mbik):
    wl = W.generate(4, 70, first=57000)
    plan = rw_plan(wl, 8, 2)
    first = plan.solve_host(wl.pose, wl.targets)
    loaded = Plan.load(plan.save())
    assert loaded.info()["wave_roles"] == 1 and loaded.info()["lanes_per_skeleton"] == 8
    got = loaded.solve_host(wl.pose, wl.targets)
    assert np.array_equal(got.view(np.uint32), first.view(np.uint32))


@pytest.mark.parametrize("cfg,n,k", [(4, 32768, 4), (5, 16384, 8), (4, 262144, 4)])
def test_wave_roles_full_size(oracle, mbik, torch_dev, cfg, n, k):
    """BASELINE sizes on the layouts the bench times (K4 / K8 at two waves per SIMD; C4's whole
    262,144-skeleton batch is the strong-scaling line's layout, where the device-memory state
    areas and their 32-bit buffer offsets are largest): whole-batch properties and oracle checks
    at the start, a third in, the middle and the last six skeletons."""
    torch, dev = torch_dev
    wl = W.generate(cfg, n)
    plan = rw_plan(wl, k, 2)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, wl.n, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    check_info(plan, k, 2)
    got = po.cpu().numpy()
    del pi, tg, po
    assert np.isfinite(got).all()
    q = got[..., :4]
    assert np.abs(np.linalg.norm(q, axis=-1) - 1).max() < 1e-5
    for first, cnt in ((0, 3), (4093, 3), (n // 3, 3), (n // 2 + 17, 3), (n - 6, 6)):
        sub = W.generate(cfg, cnt, first=first)
        ref = oracle.Oracle(sub).solve(sub.pose, sub.targets, threads=8)
        assert_parity(got[first:first + cnt], ref, f"C{cfg} wave roles full size @{first}")


def test_wave_roles_plan_in_a_group(oracle, mbik, torch_dev):
    """mbik_group_solve launches a wave-roles plan on its own (its state is in device memory)
    beside the fused launch of the classic plans."""
    torch, dev = torch_dev
    from many_bone_ik_amd.solver import Group
    wls = [W.generate(2, 20, first=58000), W.generate(4, 70, first=58100), W.generate(5, 9, first=58200)]
    plans = [Plan.from_workload(wls[0]), rw_plan(wls[1], 8, 2), rw_plan(wls[2], 4, 1)]
    ins = [torch.from_numpy(w.pose).to(dev) for w in wls]
    tgs = [torch.from_numpy(w.targets).to(dev) for w in wls]
    outs = [torch.empty_like(x) for x in ins]
    Group(plans).solve([x.data_ptr() for x in ins], [x.data_ptr() for x in tgs], [x.data_ptr() for x in outs])
    torch.cuda.synchronize()
    assert [p.info()["wave_roles"] for p in plans] == [0, 1, 1]
    for w, o in zip(wls, outs):
        assert_parity(o.cpu().numpy(), oracle.Oracle(w).solve(w.pose, w.targets, threads=8), f"group {w.topo.name}")


@pytest.mark.parametrize("cfg,n,k,spw", [(2, 70, 4, 16), (5, 40, 8, 32), (4, 50, 4, 8)])
def test_wave_roles_partly_filled_waves(oracle, mbik, cfg, n, k, spw):
    """A pinned skeletons-per-block below 64: each wave's lanes past spw idle at every barrier."""
    wl = W.generate(cfg, n, first=59000 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(k, spw, 0)
    plan.set_waves_per_simd(2)
    plan.set_wave_roles(1)
    got = plan.solve_host(wl.pose, wl.targets)
    info = plan.info()
    assert info["wave_roles"] == 1 and info["skeletons_per_block"] == spw
    assert_parity(got, ref, f"C{cfg} wave roles K={k} spw={spw}")


@pytest.mark.parametrize("cfg,k", [(4, 4), (5, 8)])
def test_wave_roles_record_handshake_has_an_exit(oracle, mbik, torch_dev, cfg, k):
    """A cooperative group's parent-side records (bone_step.h rw_record / rw_wait): the group's
    first wave posts each record it has read, and the second wave stores the next one only then.
    Test hook (mbik_plan_debug_helper): the first wave stops posting after record 1, with a 20 ms
    deadline.  The second wave gives up instead of hanging; every skeleton of the launch is written
    as a failure and flagged, the plan's status and next call report the timeout, and with the hook
    off the plan is exact again."""
    from many_bone_ik_amd import _lib
    from .test_gpu_helper_wave import _timeout_marker_ok
    torch, dev = torch_dev
    wl = W.generate(cfg, 70, first=60500 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = rw_plan(wl, k, 2)
    plan.debug_helper(1, 20000)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    flags = torch.zeros(wl.n, dtype=torch.uint8, device=dev)
    plan.solve_checked(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), flags.data_ptr())
    torch.cuda.synchronize()
    assert plan.status() == 1
    assert flags.cpu().numpy().all()
    assert _timeout_marker_ok(po.cpu().numpy())
    with pytest.raises(_lib.MbikError) as e:
        plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    assert e.value.code == _lib.MBIK_EHIP
    plan.debug_helper(-1, 0)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    torch.cuda.synchronize()
    assert plan.status() == 0
    assert_parity(po.cpu().numpy(), ref, f"C{cfg} wave roles after the handshake timeout")
