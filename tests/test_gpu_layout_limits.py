"""Layouts a plan cannot have, and what the library does then.

* A wave-roles block holds the block's targets and, for a cooperative row, one effector-global
  slot per effector of the row: the root segment's row alone takes a slot per pin, so a rig with
  many pins overflows the 160 KiB LDS.  ensure_schedule falls back to the classic layout (as for
  stabilization or 64-bit tables) instead of failing at launch, so a pinned
  mbik_plan_set_wave_roles(1) still solves and the default autotune skips nothing it can run.
  The same for constraint_mode's wave roles, whose per-wave chain stacks grow with the deepest
  pose chain.
* An autotune that fails, or that has nothing eligible to time, leaves the caller's settings as
  they were (a pinned wave-roles request survives mbik_plan_save).
* mbik_multi_solve after a failing shard: the shards before it are solved, and the root stream
  still waits for what the call queued.
Bitwise against the oracle.  Needs an MI355X: -m gpu."""
import math
import struct

import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Multi, Plan

from .test_gpu_constraint_mode import run_frames
from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def fan_rig(fingers=40, length=2, constrained=False):
    """A root bone with `fingers` chains of `length` bones, each pinned at its tip: the root
    segment has one effector per finger (a cooperative row of `fingers` slots under wave roles)."""
    parents, pins = [-1], []
    for _ in range(fingers):
        p = 0
        for _ in range(length):
            parents.append(p)
            p = len(parents) - 1
        pins.append(p)
    cons = list(range(1, len(parents))) if constrained else []
    return W.custom_topology(parents, pins, cons, cones_per_bone=2 if constrained else 0,
                             twist=(math.radians(-20), math.radians(70)) if constrained else None, iterations=6,
                             name=f"fan{fingers}x{length}")


def saved_roles_override(plan) -> int:
    """mbik_plan_save's last field (format 5): the wave-roles override."""
    return struct.unpack("<i", plan.save()[-4:])[0]


def test_many_pins_autotune_default(oracle, mbik, torch_dev):
    """40 pins: every wave-roles candidate's block exceeds the LDS.  The default autotune used to
    stop at the first of them with MBIK_EUNSUPPORTED and leave the plan pinned to it."""
    torch, dev = torch_dev
    wl = W.generate(21, 300, topo=fan_rig(40))
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    info = plan.info()
    assert info["wave_roles"] == 0
    assert info["lds_bytes_per_block"] <= 160 * 1024
    plan.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    torch.cuda.synchronize()
    assert_parity(po.cpu().numpy(), ref, "40-pin fan after the default autotune")


def test_many_pins_wave_roles_pinned_falls_back(oracle, mbik):
    wl = W.generate(22, 70, topo=fan_rig(40))
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(4, 0, 0)
    plan.set_waves_per_simd(2)
    plan.set_wave_roles(1)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["wave_roles"] == 0
    assert_parity(got, ref, "40-pin fan, wave roles pinned")
    assert saved_roles_override(plan) == 1      # the pin stays: a smaller rig would get it


def test_few_pins_keep_wave_roles(oracle, mbik):
    """The fallback is only for blocks that do not fit: 8 fingers keep the wave-roles layout."""
    wl = W.generate(23, 70, topo=fan_rig(8))
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(4, 0, 0)
    plan.set_waves_per_simd(2)
    plan.set_wave_roles(1)
    got = plan.solve_host(wl.pose, wl.targets)
    assert plan.info()["wave_roles"] == 1
    assert_parity(got, ref, "8-pin fan, wave roles")


def test_deep_constraint_mode_rig_autotunes(oracle, mbik, torch_dev):
    """constraint_mode wave roles keep a chain stack per wave (K x 64 x the deepest pose chain):
    8 fingers of 80 bones do not fit at K = 8.  The default autotune times what fits; a frame
    sequence on the tuned plan stays bitwise."""
    torch, dev = torch_dev
    topo = fan_rig(8, 80, constrained=True)
    wl = W.generate(24, 40, topo=topo)
    plan = Plan.from_workload(wl, constraint_mode=True)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    assert plan.info()["lds_bytes_per_block"] <= 160 * 1024
    # the same rig with K = 8 wave roles pinned: classic constraint_mode instead, frames bitwise
    run_frames(oracle, wl, frames=3, seed=61, lanes=8, roles=1, expect_roles=0)


def test_autotune_keeps_a_pin_it_cannot_time(oracle, mbik, torch_dev):
    """Wave roles pinned on a stabilization plan: no candidate is eligible, so nothing is timed
    and the caller's pin stands (it used to be overwritten with 0)."""
    torch, dev = torch_dev
    wl = W.generate(2, 64, first=9)
    plan = Plan.from_workload(wl, stabilization_passes=1)
    plan.set_wave_roles(1)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.empty_like(pi)
    plan.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr())
    assert saved_roles_override(plan) == 1
    assert plan.info()["wave_roles"] == 0
    ref = oracle.Oracle(wl, stabilization_passes=1).solve(wl.pose, wl.targets, threads=8)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, "stabilization plan after autotune")


def test_multi_solve_stops_at_a_failing_shard(oracle, mbik, torch_dev):
    """The second shard's plan has an unreported helper-wave timeout, so its mbik_solve fails after
    the handle queued its scatter copies (MBIK_MULTI_STAGE_ALL).  The call returns MBIK_EHIP, the
    root stream drains (it waits for the failing shard's queued copies too), the first shard's
    poses are there, and the next call, with the plan healthy again, solves everything."""
    torch, dev = torch_dev
    wl = W.generate(2, 200, first=63000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    cuts = [0, 120, 200]
    plans = [Plan(wl.topo.parents, wl.pins(), wl.constraints(), wl.pose[lo:hi], wl.cones[lo:hi], wl.twist[lo:hi],
                  iterations=wl.topo.iterations, default_damp=wl.default_damp, max_cones=wl.cones.shape[2])
             for lo, hi in zip(cuts[:-1], cuts[1:])]
    for p in plans:
        p.set_helper_wave(1)
    bad = plans[1]
    bad.debug_helper(5, 20000)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.full_like(pi, float("nan"))
    tmp = torch.empty_like(pi[120:])
    bad.solve(pi[120:].data_ptr(), tg[120:].data_ptr(), tmp.data_ptr())   # times out; reported on the next call
    torch.cuda.synchronize()
    assert bad.status() == 1
    m = Multi(plans, stage_all=True)
    st = torch.cuda.Stream(dev)
    with pytest.raises(_lib.MbikError) as e:
        m.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), st.cuda_stream)
    assert e.value.code == _lib.MBIK_EHIP
    st.synchronize()
    got = po.cpu().numpy()
    assert_parity(got[:120], ref[:120], "the shard before the failing one")
    bad.debug_helper(-1, 0)
    m.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), st.cuda_stream)
    st.synchronize()
    assert_parity(po.cpu().numpy(), ref, "the next call")
