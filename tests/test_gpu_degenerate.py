"""Degenerate inputs, GPU vs oracle: zero targets, non-finite targets and poses (write-back turns a non-finite basis into the identity,
ik_bone_3d.cpp:174-176), zero-scale and zero-length bones.  Bitwise, except that a NaN only has
to be a NaN: its payload is not part of IEEE arithmetic's contract (x86 and gfx950 produce
different default NaNs) and no comparison or branch can observe it."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

pytestmark = pytest.mark.gpu


def assert_equal_nan_aware(got, ref, what):
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), f"{what}: NaN positions differ ({gn.sum()} vs {rn.sum()})"
    g, r = got.copy(), ref.copy()
    g[gn] = 0
    r[rn] = 0
    diff = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    assert diff.size == 0, f"{what}: {len(diff)} values differ; first {diff[:5].tolist()}"


def run(oracle, wl, **kw):
    ref = oracle.Oracle(wl, **kw).solve(wl.pose, wl.targets)
    got = Plan.from_workload(wl, **kw).solve_host(wl.pose, wl.targets)
    return got, ref


@pytest.mark.parametrize("stab", [0, 1])
def test_zero_targets(oracle, mbik, stab):
    """All-zero target transforms (zero basis): degenerate target headings."""
    wl = W.generate(2, 16)
    wl.targets[:4] = 0.0
    got, ref = run(oracle, wl, stabilization_passes=stab)
    assert_equal_nan_aware(got, ref, "zero targets")


@pytest.mark.parametrize("what", ["nan_target", "inf_target", "nan_pose", "zero_scale", "huge_target"])
def test_non_finite_and_degenerate(oracle, mbik, what):
    wl = W.generate(2, 24)
    rng = np.random.default_rng(5)
    s = rng.choice(wl.n, 6, replace=False)
    if what == "nan_target":
        wl.targets[s, 1, 9] = np.nan
    elif what == "inf_target":
        wl.targets[s, 2, 0] = np.inf
    elif what == "nan_pose":
        wl.pose[s, 5, 0] = np.nan
    elif what == "zero_scale":
        wl.pose[s, 3, 7:10] = 0.0
    elif what == "huge_target":
        wl.targets[s, 0, 9:12] = 3e38
    got, ref = run(oracle, wl)
    assert_equal_nan_aware(got, ref, what)
    others = np.setdiff1d(np.arange(wl.n), s)
    assert np.isfinite(got[others]).all()


def test_zero_length_bones(oracle, mbik):
    """Coincident bone origins: the bone-direction setup's zero-vector fallbacks
    (ik_bone_3d.cpp:57-93) and zero tip headings."""
    wl = W.generate(2, 12)
    wl.pose[:, 5:9, 4:7] = 0.0
    got, ref = run(oracle, wl)
    assert_equal_nan_aware(got, ref, "zero-length bones")


def test_constraint_mode_degenerate(oracle, mbik):
    wl = W.generate(2, 12)
    wl.pose[:3, 4, 7:10] = 0.0
    wl.pose[3:5, 6, 0] = np.nan
    got, ref = run(oracle, wl, constraint_mode=True)
    assert_equal_nan_aware(got, ref, "constraint_mode degenerate")


@pytest.mark.parametrize("constraint_mode", [False, True])
def test_nonfinite_flags(mbik, constraint_mode):
    """mbik_solve_checked: the same poses as mbik_solve, plus a byte per skeleton that is 1
    exactly where a non-finite basis was written as the identity (ik_bone_3d.cpp:174-176)."""
    import torch
    dev = torch.device("cuda", 0)
    wl = W.generate(2, 40)
    bad = np.array([3, 17, 18, 39])
    wl.pose[bad, 5, 0] = np.nan  # a NaN rotation: that bone's basis is non-finite throughout
    pin = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    plain = Plan.from_workload(wl, constraint_mode=constraint_mode)
    checked = Plan.from_workload(wl, constraint_mode=constraint_mode)
    out0, out1 = torch.empty_like(pin), torch.empty_like(pin)
    flags = torch.full((wl.n,), 7, dtype=torch.uint8, device=dev)
    plain.solve(pin.data_ptr(), tg.data_ptr(), out0.data_ptr())
    checked.solve_checked(pin.data_ptr(), tg.data_ptr(), out1.data_ptr(), flags.data_ptr())
    torch.cuda.synchronize()
    assert_equal_nan_aware(out1.cpu().numpy(), out0.cpu().numpy(), "checked vs plain")
    want = np.zeros(wl.n, np.uint8)
    want[bad] = 1
    assert np.array_equal(flags.cpu().numpy(), want)
    # a sub-range: flags (like the pose buffers) are indexed from `first`
    f2 = torch.full((8,), 7, dtype=torch.uint8, device=dev)
    out2 = torch.empty_like(pin)
    checked2 = Plan.from_workload(wl, constraint_mode=constraint_mode)
    checked2.solve_checked(pin[12].data_ptr(), tg[12].data_ptr(), out2[12].data_ptr(), f2.data_ptr(), first=12, count=8)
    torch.cuda.synchronize()
    assert np.array_equal(f2.cpu().numpy(), want[12:20])


def test_selftest_math(mbik):
    """The solve's square root equals the correctly rounded sqrtf on all 2^32 inputs."""
    import ctypes
    out = (ctypes.c_uint64 * 2)()
    assert mbik.mbik_selftest_math(0, out) == 0
    assert list(out) == [0, 0]
