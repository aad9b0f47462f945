"""Heading-slot specialisation (mbik_plan_info.heading_slots, ABI 7).  When every effector has the
reference's default direction priorities (0.2, 0, 0.2) -- ik_effector_template_3d.h:45 -- the plan
launches kernels built for that heading set (origin, +/-x, +/-z as compile-time slots); any other
priorities run the kernels that test each effector's slots at run time.  Both families must be
bitwise equal to the oracle in every layout they serve: one wave per SIMD in each state
placement, two waves with and without split-exchange headings, the helper wave, stabilization
(always the run-time family) and groups mixing both.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

from .test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu

DEFAULT_SLOTS = 0x67

PRIORITIES = {
    "default": None,                                  # the generator's (0.2, 0, 0.2) for every pin
    "all_axes": (0.2, 0.1, 0.2),                     # 0x7f: uniform, but not the specialised set
    "y_only": (0.0, 0.5, 0.0),                       # 0x19
    "mixed": "mixed",                                # per pin: default, none, all three axes
}


def workload(cfg, n, prio, first):
    wl = W.generate(cfg, n, first=first)
    P = wl.pin_priority.shape[0]
    if prio == "mixed":
        choices = np.array([[0.2, 0.0, 0.2], [0.0, 0.0, 0.0], [0.3, 0.2, 0.1]], np.float32)
        wl.pin_priority = choices[np.arange(P) % 3].copy()
    elif prio is not None:
        wl.pin_priority = np.tile(np.array(prio, np.float32), (P, 1))
    return wl


@pytest.mark.parametrize("name", list(PRIORITIES))
def test_heading_slots_reported(mbik, name):
    wl = workload(2, 4, PRIORITIES[name], 0)
    info = Plan.from_workload(wl).info()
    assert info["heading_slots"] == (DEFAULT_SLOTS if name == "default" else 0)


def test_one_non_default_pin_selects_runtime_slots(mbik):
    wl = W.generate(5, 2)
    assert Plan.from_workload(wl).info()["heading_slots"] == DEFAULT_SLOTS
    wl.pin_priority = wl.pin_priority.copy()
    wl.pin_priority[-1, 1] = 0.05                    # the last finger also weighs its y axis
    assert Plan.from_workload(wl).info()["heading_slots"] == 0


# (cfg, n, lanes, interval, staging, placement, waves, helper): the layouts the autotune picks for
# C2-C5 plus the other state placements of each build
LAYOUTS = [
    (2, 48, 4, 1, 1, 0, 1, 1),
    (2, 48, 4, 1, 1, 0, 1, 0),
    (3, 48, 4, 4, 4, 1, 2, 0),
    (3, 48, 4, 2, 0, 1, 1, 0),
    (4, 16, 4, 1, 4, 2, 2, 0),
    (4, 16, 4, 1, 0, 2, 2, 0),
    (4, 16, 8, 4, 1, 1, 1, 0),
    (5, 6, 8, 1, 4, 2, 2, 0),
    (5, 6, 8, 2, 2, 2, 1, 0),
    (5, 6, 16, 1, 4, 1, 2, 0),
]


@pytest.mark.parametrize("layout", LAYOUTS, ids=lambda l: "C{}_K{}_i{}_st{}_pl{}_w{}_h{}".format(l[0], *l[2:]))
@pytest.mark.parametrize("name", list(PRIORITIES))
def test_heading_slot_families_bitwise_vs_oracle(oracle, mbik, layout, name):
    cfg, n, lanes, interval, staging, placement, waves, helper = layout
    wl = workload(cfg, n, PRIORITIES[name], 41000 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl)
    plan.set_layout(lanes, 0, interval)
    plan.set_heading_staging(staging)
    plan.set_locals_placement(placement)
    plan.set_waves_per_simd(waves)
    plan.set_helper_wave(helper)
    got = plan.solve_host(wl.pose, wl.targets)
    info = plan.info()
    assert info["heading_slots"] == (DEFAULT_SLOTS if name == "default" else 0)
    assert info["state_placement"] == placement and info["waves_per_simd"] == waves
    assert_parity(got, ref, f"C{cfg} {name} layout {layout}")


@pytest.mark.parametrize("name", ["default", "all_axes"])
def test_heading_slots_with_stabilization(oracle, mbik, name):
    wl = workload(2, 24, PRIORITIES[name], 42000)
    ref = oracle.Oracle(wl, stabilization_passes=2).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, stabilization_passes=2)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C2 {name} stabilization")


def test_group_mixes_both_families(oracle, mbik):
    """A fused group launch runs every plan through the run-time-slot build, whichever family its
    own launches use."""
    import torch
    from many_bone_ik_amd.solver import Group
    dev = torch.device("cuda", 0)
    wls = [workload(2, 20, None, 43000), workload(3, 24, PRIORITIES["mixed"], 43100), workload(5, 4, None, 43200)]
    plans = [Plan.from_workload(w) for w in wls]
    assert [p.info()["heading_slots"] for p in plans] == [DEFAULT_SLOTS, 0, DEFAULT_SLOTS]
    ins = [torch.from_numpy(w.pose).to(dev) for w in wls]
    tgs = [torch.from_numpy(w.targets).to(dev) for w in wls]
    outs = [torch.empty_like(x) for x in ins]
    Group(plans).solve([x.data_ptr() for x in ins], [x.data_ptr() for x in tgs], [x.data_ptr() for x in outs])
    torch.cuda.synchronize()
    for w, o in zip(wls, outs):
        assert_parity(o.cpu().numpy(), oracle.Oracle(w).solve(w.pose, w.targets, threads=8), f"group {w.topo.name}")
