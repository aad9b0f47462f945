"""Plan serialisation (mbik_plan_save / mbik_plan_load, SURVEY.md §5 "plan serialisable to a
flat binary"): a loaded plan solves bitwise like the saved one -- setup tables rebuilt on the
GPU, layout overrides and constraint_mode's persistent node caches included -- and corrupt or
truncated buffers are refused."""
import ctypes as C

import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n", [(1, 1), (2, 48), (3, 32), (4, 8), (5, 4)])
def test_loaded_plan_solves_bitwise(oracle, mbik, cfg, n):
    wl = W.generate(cfg, n, first=7)
    a = Plan.from_workload(wl)
    a.set_layout(0, 3, 2)                       # a non-default layout must survive the round trip
    data = a.save()
    b = Plan.load(data)
    got_a = a.solve_host(wl.pose, wl.targets)
    got_b = b.solve_host(wl.pose, wl.targets)
    keys = ("skeletons_per_block", "checkpoint_interval", "bone_count", "pin_count", "lanes_per_skeleton")
    assert {k: b.info()[k] for k in keys} == {k: a.info()[k] for k in keys}
    assert np.array_equal(got_a.view(np.uint32), got_b.view(np.uint32))
    assert_parity(got_b, oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8), f"C{cfg} loaded plan")
    # saving the loaded plan gives the same bytes
    assert b.save() == data


def test_table_addressing_override_survives(oracle, mbik):
    """mbik_plan_set_table_addressing(1) is one of the saved layout overrides (format 2): the
    loaded plan still runs the 64-bit-index kernel -- bitwise like the original -- and so still
    refuses placement 1, which needs the 32-bit form."""
    wl = W.generate(2, 24, first=11)
    a = Plan.from_workload(wl)
    a.set_table_addressing(1)
    data = a.save()
    b = Plan.load(data)
    assert b.save() == data
    got = b.solve_host(wl.pose, wl.targets)
    assert np.array_equal(got.view(np.uint32), a.solve_host(wl.pose, wl.targets).view(np.uint32))
    assert_parity(got, oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8), "loaded 64-bit-table plan")
    b.set_locals_placement(1)
    with pytest.raises(_lib.MbikError):
        b.solve_host(wl.pose, wl.targets)


def test_rebuilt_setup_tables_survive(mbik):
    import torch
    wl = W.generate(5, 6)
    other = W.generate(5, 6, first=900)          # different setup poses / cones
    a = Plan.from_workload(wl)
    dev = torch.device("cuda", 0)
    sp = torch.from_numpy(other.pose).to(dev)
    cn = torch.from_numpy(np.ascontiguousarray(other.cones)).to(dev)
    tw = torch.from_numpy(np.ascontiguousarray(other.twist)).to(dev)
    a.rebuild_setup(sp.data_ptr(), cn.data_ptr(), tw.data_ptr())
    b = Plan.load(a.save())
    for ta, tb in zip(a.setup_tables(), b.setup_tables()):
        assert np.array_equal(ta.view(np.uint8), tb.view(np.uint8))
    ga = a.solve_host(wl.pose, wl.targets)
    gb = b.solve_host(wl.pose, wl.targets)
    assert np.array_equal(ga.view(np.uint32), gb.view(np.uint32))


def test_constraint_mode_node_caches_survive(mbik):
    """constraint_mode frames depend on the node caches earlier frames left: a
    plan saved after two frames and loaded elsewhere continues exactly like the original."""
    wl = W.generate(2, 16, first=3)
    a = Plan.from_workload(wl, constraint_mode=True)
    pose = wl.pose
    for _ in range(2):
        pose = a.solve_host(pose, wl.targets)
    data = a.save()
    b = Plan.load(data)
    assert b.save() == data                       # node caches and dirty words restored byte for byte
    for _ in range(2):
        ga = a.solve_host(pose, wl.targets)
        gb = b.solve_host(pose, wl.targets)
        assert np.array_equal(ga.view(np.uint32), gb.view(np.uint32))
        pose = ga
    assert a.save() == b.save()


def test_corrupt_buffers_are_refused(mbik):
    wl = W.generate(2, 4)
    data = Plan.from_workload(wl).save()
    L = _lib.load()
    h = C.c_void_p()
    for bad in (b"", b"MBIKPLAN", b"X" + data[1:], data[:-1], data[: len(data) // 2]):
        rc = L.mbik_plan_load(bad, len(bad), 0, C.byref(h))
        assert rc == _lib.MBIK_EINVAL and not h.value
    size = C.c_uint64(0)
    p = Plan.from_workload(wl)
    small = C.create_string_buffer(16)
    assert L.mbik_plan_save(p.h, small, 16, C.byref(size)) == _lib.MBIK_EINVAL
    assert size.value == len(data)
