"""Results do not depend on the launch layout (mbik_plan_set_layout): lanes per skeleton,
skeletons per block and the checkpoint interval of the iteration-start globals kept in
LDS.  Every layout is bitwise equal to the oracle.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n", [(1, 8), (2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("interval", [2, 3, 1 << 20])
@pytest.mark.parametrize("lanes,spw", [(0, 0), (0, 3), (4, 0), (1, 5)])
def test_layouts_bitwise_vs_oracle(oracle, mbik, cfg, n, interval, lanes, spw):
    wl = W.generate(cfg, n, first=5000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(lanes, spw, interval)
    got = plan.solve_host(wl.pose, wl.targets)
    info = plan.info()
    assert spw == 0 or info["skeletons_per_block"] <= spw
    assert_parity(got, ref, f"C{cfg} interval={interval} lanes={lanes} spw={spw}")


def test_layout_with_stabilization(oracle, mbik):
    wl = W.generate(1, 16, first=77)
    ref = oracle.Oracle(wl, stabilization_passes=2).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=2)
    plan.set_layout(0, 7, 3)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, "C1 stab interval=3")


def test_auto_layout_of_a_large_launch_is_exact(oracle, mbik):
    """A launch larger than the chip holds switches to the residency layout; spot-check it."""
    import torch
    wl = W.generate(5, 16384)
    plan = Plan.from_workload(wl)
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, wl.n, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    got = po.cpu().numpy()
    for first in (0, 8191, 16380):
        sub = W.generate(5, 4, first=first)
        ref = oracle.Oracle(sub).solve(sub.pose, sub.targets, threads=8)
        assert_parity(got[first:first + 4], ref, f"C5 auto layout @{first}")


def test_layout_argument_checks(mbik):
    wl = W.generate(3, 2)
    plan = Plan.from_workload(wl)
    for args in [(3, 0, 0), (0, 65, 0), (0, 0, -1)]:
        with pytest.raises(_lib.MbikError) as e:
            plan.set_layout(*args)
        assert e.value.code == _lib.MBIK_EINVAL


def test_autotune_keeps_results(oracle, mbik):
    import torch
    wl = W.generate(2, 512, first=9000)
    plan = Plan.from_workload(wl)
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), stream=st)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), stream=st)
    torch.cuda.synchronize()
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    assert_parity(po.cpu().numpy(), ref, "C2 after autotune")


@pytest.mark.parametrize("constraint_mode", [False, True])
def test_autotune_refuses_overlapping_buffers(mbik, constraint_mode):
    """Every candidate layout is timed on the same input, so pose_in and pose_out must not
    overlap (mbik.h); an in-place call would advance the caller's pose once per timed run."""
    import torch
    wl = W.generate(3, 64)
    plan = Plan.from_workload(wl, constraint_mode=constraint_mode)
    pi = torch.from_numpy(wl.pose).to("cuda:0")
    tg = torch.from_numpy(wl.targets).to("cuda:0")
    for out_ptr in (pi.data_ptr(), pi[1:].data_ptr()):
        with pytest.raises(_lib.MbikError) as e:
            plan.autotune(pi.data_ptr(), tg.data_ptr(), out_ptr)
        assert e.value.code == _lib.MBIK_EINVAL
    before = pi.cpu().numpy()
    assert np.array_equal(before, wl.pose)


@pytest.mark.parametrize("cfg,n", [(2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("stab", [0, 2])
@pytest.mark.parametrize("lanes", [0, 16])
@pytest.mark.parametrize("staging", [0, 2, 3])
def test_unstaged_headings_bitwise_vs_oracle(oracle, mbik, cfg, n, stab, lanes, staging):
    """mbik_plan_set_heading_staging(0): every lane of a multi-effector segment's group solves
    the segment alone (no LDS staging); (2): only the translating root segments are staged;
    (3): only segments with two or more effectors; still bitwise equal to the oracle."""
    wl = W.generate(cfg, n, first=9000)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    plan.set_layout(lanes, 0, 0)
    plan.set_heading_staging(staging)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["heading_staging"] == staging
    assert_parity(got, ref, f"C{cfg} staging={staging} lanes={lanes} stab={stab}")


def test_staging_argument_check(mbik):
    plan = Plan.from_workload(W.generate(3, 2))
    with pytest.raises(_lib.MbikError):
        plan.set_heading_staging(6)
    plan.set_heading_staging(-1)


@pytest.mark.parametrize("cfg,n", [(2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("staging", [4, 5])
@pytest.mark.parametrize("placement", [0, 1, 2])
@pytest.mark.parametrize("lanes", [0, 16])
def test_split_exchange_bitwise_vs_oracle(oracle, mbik, cfg, n, staging, placement, lanes):
    """mbik_plan_set_heading_staging(4 | 5) in the two-wave build: a multi-effector segment's
    lanes build alternate effectors' headings and read each other's lane to lane, every lane
    summing all of them in order (5: translating roots staged in memory instead); bitwise."""
    wl = W.generate(cfg, n, first=31000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(lanes, 0, 0)
    plan.set_waves_per_simd(2)
    plan.set_locals_placement(placement)
    plan.set_heading_staging(staging)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["heading_staging"] == staging
    assert_parity(got, ref, f"C{cfg} staging={staging} placement={placement} lanes={lanes}")


@pytest.mark.parametrize("cfg,n", [(4, 16), (5, 6)])
def test_split_exchange_in_one_wave_build_solves_alone(oracle, mbik, cfg, n):
    """The one-wave build has no split-exchange code: staging 4 / 5 there solve those segments
    alone (as 0 / 2) and stay exact; a group with a split-exchange plan launches it on its own."""
    from many_bone_ik_amd.solver import Group
    import torch
    wl = W.generate(cfg, n, first=32000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_heading_staging(4)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} staging 4, one wave")
    plan.set_waves_per_simd(2)
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    wl3 = W.generate(3, 24, first=50)
    plan3 = Plan.from_workload(wl3)
    pi3 = torch.from_numpy(wl3.pose).to(dev)
    tg3 = torch.from_numpy(wl3.targets).to(dev)
    po3 = torch.empty_like(pi3)
    grp = Group([plan, plan3])
    grp.solve([pi.data_ptr(), pi3.data_ptr()], [tg.data_ptr(), tg3.data_ptr()], [po.data_ptr(), po3.data_ptr()])
    torch.cuda.synchronize()
    assert_parity(po.cpu().numpy(), ref, f"group: C{cfg} split-exchange plan")
    assert_parity(po3.cpu().numpy(), oracle.Oracle(wl3).solve(wl3.pose, wl3.targets, threads=8), "group: LDS plan")


@pytest.mark.parametrize("cfg,n", [(1, 8), (2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("staging", [1, 0, 2, 3])
@pytest.mark.parametrize("stab", [0, 2])
@pytest.mark.parametrize("placement", [1, 2])
def test_state_in_hbm_bitwise_vs_oracle(oracle, mbik, cfg, n, staging, stab, placement):
    """mbik_plan_set_locals_placement(1 | 2): the bone locals (1) or the whole per-skeleton
    state (2, staged headings included) live in device memory during the launch; lanes
    exchange them through L2 across the row and wave barriers; bitwise equal."""
    wl = W.generate(cfg, n, first=12000)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    plan.set_locals_placement(placement)
    plan.set_heading_staging(staging)
    got = plan.solve_host(wl.pose, wl.targets)
    assert_parity(got, ref, f"C{cfg} state placement {placement} staging={staging} stab={stab}")
    plan.set_locals_placement(0)                          # back to LDS: same bits
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} locals back in LDS")


@pytest.mark.parametrize("placement", [1, 2])
def test_state_in_hbm_subrange_and_group(oracle, mbik, placement):
    """A subrange launch indexes the HBM locals by absolute skeleton; a group with such a plan
    launches it on its own and the results stay exact."""
    from many_bone_ik_amd.solver import Group
    wl = W.generate(2, 40, first=300)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_locals_placement(placement)
    import torch
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.zeros_like(pi)
    plan.solve(pi[10].data_ptr(), tg[10].data_ptr(), po[10].data_ptr(), 10, 20)
    torch.cuda.synchronize()
    assert_parity(po[10:30].cpu().numpy(), ref[10:30], "HBM locals subrange")
    wl3 = W.generate(3, 24, first=50)
    ref3 = oracle.Oracle(wl3).solve(wl3.pose, wl3.targets, threads=8)
    plan3 = Plan.from_workload(wl3)
    grp = Group([plan, plan3])
    pi3 = torch.from_numpy(wl3.pose).to(dev)
    tg3 = torch.from_numpy(wl3.targets).to(dev)
    po1, po3 = torch.empty_like(pi), torch.empty_like(pi3)
    grp.solve([pi.data_ptr(), pi3.data_ptr()], [tg.data_ptr(), tg3.data_ptr()], [po1.data_ptr(), po3.data_ptr()])
    torch.cuda.synchronize()
    assert_parity(po1.cpu().numpy(), ref, "group: HBM-locals plan")
    assert_parity(po3.cpu().numpy(), ref3, "group: LDS plan")


@pytest.mark.parametrize("cfg,n", [(2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("placement", [0, 1, 2])
def test_two_waves_per_simd_bitwise_vs_oracle(oracle, mbik, cfg, n, placement):
    """mbik_plan_set_waves_per_simd(2): the 256-register build (spilling to scratch) computes
    the same bits."""
    wl = W.generate(cfg, n, first=15000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_waves_per_simd(2)
    plan.set_locals_placement(placement)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} 2 waves/SIMD placement {placement}")


@pytest.mark.parametrize("cfg,n", [(2, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("waves", [1, 2])
def test_table_addressing_64bit_bitwise_vs_oracle(oracle, mbik, cfg, n, waves):
    """mbik_plan_set_table_addressing(1): the instantiation with 64-bit table indices -- the
    one plans whose setup tables reach 4 GiB run -- computes the same bits, placements 1 and 2
    refuse it, and a fused group launches such a plan on its own."""
    wl = W.generate(cfg, n, first=21000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_table_addressing(1)
    plan.set_waves_per_simd(waves)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} 64-bit table indices, {waves} waves/SIMD")
    plan.set_locals_placement(1)
    with pytest.raises(_lib.MbikError):
        plan.solve_host(wl.pose, wl.targets)
    plan.set_locals_placement(0)
    if waves == 1 and cfg == 2:
        import torch
        from many_bone_ik_amd.solver import Group
        wl3 = W.generate(3, 24, first=77)
        ref3 = oracle.Oracle(wl3).solve(wl3.pose, wl3.targets, threads=8)
        plan3 = Plan.from_workload(wl3)
        grp = Group([plan, plan3])
        dev = torch.device("cuda", 0)
        pi, pi3 = torch.from_numpy(wl.pose).to(dev), torch.from_numpy(wl3.pose).to(dev)
        tg, tg3 = torch.from_numpy(wl.targets).to(dev), torch.from_numpy(wl3.targets).to(dev)
        po, po3 = torch.empty_like(pi), torch.empty_like(pi3)
        grp.solve([pi.data_ptr(), pi3.data_ptr()], [tg.data_ptr(), tg3.data_ptr()], [po.data_ptr(), po3.data_ptr()])
        torch.cuda.synchronize()
        assert_parity(po.cpu().numpy(), ref, "group: 64-bit-table plan")
        assert_parity(po3.cpu().numpy(), ref3, "group: 32-bit-table plan")
    with pytest.raises(_lib.MbikError):
        plan.set_table_addressing(2)


def test_tables_past_4gib_use_64bit_indices(oracle, mbik):
    """A placement-0 plan whose constraint table passes 4 GiB (the C5 rig's CF is 60.5 KB per
    skeleton: 72,000 skeletons make 4.36 GB) solves through the 64-bit-index kernel by itself,
    and placement 1 refuses it.  The batch repeats 64 distinct skeletons, so the oracle's
    results for those 64 check the first and the last 64 (the latter read table offsets past
    2^32 bytes)."""
    import dataclasses
    base = W.generate(5, 64, first=333)
    n = 72000
    rep = n // 64
    wl = dataclasses.replace(base, n=n, pose=np.tile(base.pose, (rep, 1, 1)), targets=np.tile(base.targets, (rep, 1, 1)),
                             cones=np.tile(base.cones, (rep, 1, 1, 1)), twist=np.tile(base.twist, (rep, 1, 1)))
    assert wl.pose.shape[0] == n and 199 * (14 + 31 * 2) * n * 4 > 2 ** 32
    ref = oracle.Oracle(base).solve(base.pose, base.targets, threads=8)
    plan = Plan.from_workload(wl)
    got = plan.solve_host(wl.pose, wl.targets)
    assert_parity(got[:64], ref, "C5 x 72,000 (tables > 4 GiB): first 64")
    assert_parity(got[n - 64:], ref, "C5 x 72,000 (tables > 4 GiB): last 64")
    plan.set_locals_placement(1)
    with pytest.raises(_lib.MbikError):
        plan.solve_host(base.pose[:1], base.targets[:1])


def test_waves_argument_check(mbik):
    plan = Plan.from_workload(W.generate(3, 2))
    with pytest.raises(_lib.MbikError):
        plan.set_waves_per_simd(3)


@pytest.mark.parametrize("cfg,n,pin", [(3, 65536, None), (5, 16384, (8, 8, 2, 4, 2, 2)), (5, 16384, (8, 8, 1, 0, 2, 2)),
                                       (5, 16384, (8, 8, 1, 4, 2, 2)),
                                       (4, 32768, None), (4, 262144, (4, 16, 1, 4, 2, 2))])
def test_tuned_full_size_layouts_are_exact(oracle, mbik, cfg, n, pin):
    """Full-size launches on the layouts autotune picks for them (C3, and C4 at its 32,768
    skeletons per GPU: autotuned here; C5: the layout its autotune picks, pinned -- 8 lanes x 8,
    checkpoint every 2nd bone, split-exchange headings (staging 4), all state in device memory,
    two waves per SIMD -- the same with a checkpoint at every bone (the layout round 3's C5
    bench line ran, K8_s8_i1_st4_pl2_w2), and round 2's unstaged one; C4's whole 262,144-skeleton batch
    of BASELINE configs[3] on one GPU: the strong-scaling layout, pinned -- 4 lanes x 16,
    split-exchange, all state in device memory (each area < 4 GiB: the buffer-resource guard),
    two waves per SIMD); oracle
    spot checks at the start, middle and end of the batch.  C4 is the multi-segment branching
    rig of ik_bone_segment_3d.cpp:210-225 (11 segments, post-order recursion)."""
    import torch
    wl = W.generate(cfg, n)
    plan = Plan.from_workload(wl)
    dev = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    if pin is None:
        plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    else:
        lanes, spw, interval, staging, placement, waves = pin
        plan.set_layout(lanes, spw, interval)
        plan.set_heading_staging(staging)
        plan.set_locals_placement(placement)
        plan.set_waves_per_simd(waves)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    torch.cuda.synchronize()
    got = po.cpu().numpy()
    info = plan.info()
    if pin is not None:
        assert (info["lanes_per_skeleton"], info["state_placement"], info["waves_per_simd"]) == (pin[0], pin[4], pin[5])
    # whole batch: finite, unit rotations (size-independent properties)
    assert np.isfinite(got).all(), f"C{cfg} x {n}: non-finite output"
    qn = np.linalg.norm(got[..., :4].astype(np.float64), axis=-1)
    assert np.abs(qn - 1.0).max() < 1e-5, f"C{cfg} x {n}: non-unit rotation"
    spots = (0, n // 2 - 3, n - 6) if n <= 65536 else (0, n // 3 + 1, n // 2 - 3, 2 * n // 3 + 5, n - 22, n - 6)
    for first in spots:
        sub = W.generate(cfg, 6, first=first)
        ref = oracle.Oracle(sub).solve(sub.pose, sub.targets, threads=8)
        assert_parity(got[first:first + 6], ref, f"C{cfg} tuned layout {info} @{first}")


@pytest.mark.parametrize("waves", [1, 2])
def test_state_in_hbm_reads_rebuilt_setup_tables(oracle, mbik, waves):
    """Placement 2 reads a skeleton-tiled copy of the per-skeleton tables (DevPlan::row_n):
    after mbik_plan_rebuild_setup the copy is rebuilt, so the solve follows the new rest poses,
    cones and twist like a plan created from them (bitwise, 19 skeletons: a ragged last tile)."""
    import torch
    wl = W.generate(5, 19, first=40)
    other = W.generate(5, 19, first=900)                     # other rest poses, cones, twist
    plan = Plan.from_workload(wl)
    plan.set_locals_placement(2)
    plan.set_waves_per_simd(waves)
    first = plan.solve_host(wl.pose, wl.targets)             # builds the tiled copy of wl's tables
    assert_parity(first, oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8), "placement 2 before rebuild")
    dev = torch.device("cuda", 0)
    sp = torch.from_numpy(other.pose).to(dev)
    cn = torch.from_numpy(np.ascontiguousarray(other.cones)).to(dev)
    tw = torch.from_numpy(np.ascontiguousarray(other.twist)).to(dev)
    plan.rebuild_setup(sp.data_ptr(), cn.data_ptr(), tw.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = plan.solve_host(wl.pose, wl.targets)
    fresh = Plan.from_workload(other)
    want = fresh.solve_host(wl.pose, wl.targets)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert not np.array_equal(got.view(np.uint32), first.view(np.uint32))


@pytest.mark.parametrize("cfg,n,lanes", [(5, 12, 8), (5, 12, 4), (4, 16, 4), (2, 24, 2)])
@pytest.mark.parametrize("stab", [0, 2])
@pytest.mark.parametrize("placement,waves", [(0, 1), (1, 2), (2, 2)])
def test_packed_levels_bitwise_vs_oracle(oracle, mbik, cfg, n, lanes, stab, placement, waves):
    """A sibling level wider than the lane count is packed (build_schedule, SCHED_CHAIN): each
    lane runs its own sequence of segments back to back, balanced by estimated step work (C5's
    16 fingers of 6-14 bones on 8 or 4 lanes); sibling segments are independent, so the results
    stay bitwise equal."""
    wl = W.generate(cfg, n, first=33000)
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    plan.set_layout(lanes, 0, 0)
    plan.set_locals_placement(placement)
    plan.set_waves_per_simd(waves)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["lanes_per_skeleton"] == lanes
    assert_parity(got, ref, f"C{cfg} packed levels lanes={lanes} stab={stab} placement={placement} waves={waves}")
