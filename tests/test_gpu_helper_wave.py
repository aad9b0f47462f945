"""The helper wave (mbik_plan_set_helper_wave): a second wave per block runs the global pass
and computes each bone-step's parent-side work one step ahead into an LDS ring; the solving
wave reads it instead of computing it.  Same operations on the same inputs, so every result
stays bitwise equal to the oracle and to the one-wave launch.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu
RING_BYTES = 4 * 18 * 64 * 16 + 32   # csrc/kernels.h: kHelpRingBytes (kHelpSlots x kHelpF4 float4 per lane + counters)


def _helper_fits(info):
    return info["lds_bytes_per_block"] + RING_BYTES <= 160 * 1024


def _dev():
    import torch
    return torch, torch.device("cuda", 0)


@pytest.mark.parametrize("cfg,n", [(1, 8), (2, 48), (3, 48), (4, 16), (5, 6)])
@pytest.mark.parametrize("lanes,spw", [(0, 0), (0, 3), (1, 5), (4, 0)])
def test_helper_wave_bitwise_vs_oracle(oracle, mbik, cfg, n, lanes, spw):
    """Every config and lane layout, including partial blocks (spw not dividing n) and lanes
    whose segment is shorter than the row's longest (idle steps in the shared sequence)."""
    wl = W.generate(cfg, n, first=21000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(lanes, spw, 0)
    plan.set_helper_wave(1)
    got = plan.solve_host(wl.pose, wl.targets)
    info = plan.info()
    # (a block whose LDS leaves no room for the ring launches without the helper)
    assert info["helper_wave"] == (1 if _helper_fits(info) else 0)
    assert_parity(got, ref, f"C{cfg} helper lanes={lanes} spw={spw}")


@pytest.mark.parametrize("cfg,n", [(2, 96), (5, 6)])
@pytest.mark.parametrize("interval", [2, 1 << 20])
def test_helper_wave_sparse_checkpoints(oracle, mbik, cfg, n, interval):
    """With sparse checkpoints the helper rebuilds the parent's global through unsolved
    ancestors (the SR_PARENT_GLOBAL path): still bitwise."""
    wl = W.generate(cfg, n, first=22000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(0, 0, interval)
    plan.set_helper_wave(1)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} helper interval={interval}")


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_helper_wave_segment_solve(oracle, mbik, cfg):
    """mbik_segment_solve restricts the rows' tasks (seg_lo..seg_hi): both waves walk the same
    restricted sequence."""
    torch, dev = _dev()
    wl = W.generate(cfg, 8)
    o = oracle.Oracle(wl)
    plan = Plan.from_workload(wl)
    plan.set_helper_wave(1)
    nseg = plan.info()["segment_count"]
    for seg in sorted({0, nseg // 2, nseg - 1}):
        ref = o.segment_solve(seg, wl.pose, wl.targets)
        pose = torch.from_numpy(wl.pose.copy()).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, pose.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(pose.cpu().numpy(), ref, f"C{cfg} helper segment {seg}")


def test_helper_wave_full_c2_batch(oracle, mbik):
    """BASELINE configs[1] at its size: the whole 4,096-skeleton batch with the helper equals
    the one-wave launch bit for bit, and the oracle at both ends and the middle."""
    torch, dev = _dev()
    wl = W.generate(2, 4096)
    plan = Plan.from_workload(wl)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for h in (0, 1):
        plan.set_helper_wave(h)
        po = torch.empty_like(pi)
        plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, wl.n, st)
        torch.cuda.synchronize()
        assert plan.info()["helper_wave"] == h
        outs.append(po.cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    for first in (0, 2047, 4092):
        sub = W.generate(2, 4, first=first)
        ref = oracle.Oracle(sub).solve(sub.pose, sub.targets, threads=4)
        assert_parity(outs[1][first:first + 4], ref, f"C2 helper @{first}")


@pytest.mark.parametrize("what", ["stabilization", "placement1", "placement2", "two_waves"])
def test_helper_wave_ignored_where_it_does_not_serve(oracle, mbik, what):
    """Layouts the helper does not serve launch without it (info says 0) and stay exact."""
    wl = W.generate(2, 24, first=23000)
    stab = 2 if what == "stabilization" else 0
    ref = oracle.Oracle(wl, stabilization_passes=stab).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=stab)
    if what.startswith("placement"):
        plan.set_locals_placement(int(what[-1]))
    if what == "two_waves":
        plan.set_waves_per_simd(2)
    plan.set_helper_wave(1)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["helper_wave"] == 0
    assert_parity(got, ref, f"helper ignored: {what}")


def test_helper_wave_autotune_and_save(oracle, mbik):
    """Automatic (-1): autotune times the fully resident launch without and with the helper and
    keeps one; a saved plan keeps that choice (format 4), and both solve the same bits."""
    torch, dev = _dev()
    wl = W.generate(2, 1024, first=24000)
    plan = Plan.from_workload(wl)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.set_helper_wave(-1)
    plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), stream=st)
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), stream=st)
    torch.cuda.synchronize()
    chosen = plan.info()["helper_wave"]
    assert chosen in (0, 1)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    assert_parity(po.cpu().numpy(), ref, f"C2 after autotune (helper {chosen})")
    for forced in (1, 0):
        plan.set_helper_wave(forced)
        loaded = Plan.load(plan.save())
        got = loaded.solve_host(wl.pose, wl.targets)
        assert loaded.info()["helper_wave"] == forced
        assert_parity(got, ref, f"loaded plan, helper {forced}")
        loaded.close()


def test_helper_wave_argument_check(mbik):
    plan = Plan.from_workload(W.generate(3, 2))
    for bad in (2, -2):
        with pytest.raises(_lib.MbikError) as e:
            plan.set_helper_wave(bad)
        assert e.value.code == _lib.MBIK_EINVAL
    plan.set_helper_wave(-1)


def _timeout_marker_ok(out, ref_shape_bones_in_list=None):
    """write_help_timeout: identity rotation, NaN position, unit scale for every solved bone."""
    q, o, sc = out[..., 0:4], out[..., 4:7], out[..., 7:10]
    return (np.all(q == np.array([0, 0, 0, 1], np.float32)) and np.isnan(o).all() and np.all(sc == 1.0))


def test_helper_timeout_is_visible_per_plan(oracle, mbik):
    """VERDICT r3 item 3 / ADVICE r3: a helper wave that stops producing records (test hook:
    mbik_plan_debug_helper drops record 5, 20 ms deadline) makes its partner give up; every
    skeleton of the launch is written as a failure and flagged by mbik_solve_checked, the plan's
    status shows the timeout, its next asynchronous call returns MBIK_EHIP once, and a second plan
    solving concurrently on another stream sees none of it and stays bitwise exact."""
    torch, dev = _dev()
    wl = W.generate(2, 256, first=25000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    a, b = Plan.from_workload(wl), Plan.from_workload(wl)
    for p in (a, b):
        p.set_helper_wave(1)
    a.debug_helper(5, 20000)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    oa, ob = torch.empty_like(pi), torch.empty_like(pi)
    fa = torch.zeros(wl.n, dtype=torch.uint8, device=dev)
    fb = torch.ones(wl.n, dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    a.solve_checked(pi.data_ptr(), tg.data_ptr(), oa.data_ptr(), fa.data_ptr(), stream=sa.cuda_stream)
    b.solve_checked(pi.data_ptr(), tg.data_ptr(), ob.data_ptr(), fb.data_ptr(), stream=sb.cuda_stream)
    torch.cuda.synchronize()
    assert a.info()["helper_wave"] == 1 and b.info()["helper_wave"] == 1
    assert a.status() == 1 and b.status() == 0
    got_a = oa.cpu().numpy()
    assert fa.cpu().numpy().all(), "a timed-out launch must flag every skeleton"
    assert _timeout_marker_ok(got_a)
    assert not fb.cpu().numpy().any()
    assert_parity(ob.cpu().numpy(), ref, "concurrent plan on another stream")
    # the next asynchronous call reports it (once, without launching), then the plan works again
    with pytest.raises(_lib.MbikError) as e:
        a.solve(pi.data_ptr(), tg.data_ptr(), oa.data_ptr())
    assert e.value.code == _lib.MBIK_EHIP and "timed out" in str(e.value)
    assert a.status() == 0
    a.debug_helper(-1, 0)
    a.solve(pi.data_ptr(), tg.data_ptr(), oa.data_ptr())
    torch.cuda.synchronize()
    assert a.status() == 0
    assert_parity(oa.cpu().numpy(), ref, "the plan after its timeout was reported")
    # the synchronous call reports its own launch's timeout
    a.debug_helper(0, 20000)
    with pytest.raises(_lib.MbikError) as e:
        a.solve_host(wl.pose, wl.targets)
    assert e.value.code == _lib.MBIK_EHIP
    assert a.status() == 0 and b.status() == 0
    a.debug_helper(-1, 0)
    assert_parity(a.solve_host(wl.pose, wl.targets), ref, "solve_host after the timeout")


def test_helper_debug_hook_argument_check(mbik):
    plan = Plan.from_workload(W.generate(3, 2))
    for args in ((-2, 0), (0, -1)):
        with pytest.raises(_lib.MbikError) as e:
            plan.debug_helper(*args)
        assert e.value.code == _lib.MBIK_EINVAL
    assert plan.status() == 0
