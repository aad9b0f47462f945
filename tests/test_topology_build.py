"""GPU-side topology build (csrc/topo.h): the recursion-free builder one GPU
thread runs per rig must produce build_topology's tables exactly.  Here (no GPU) the same
topo.h code runs on the host (mbik_selftest_topology with device -1) over C1-C5, the edge
topologies, random rigs and invalid descriptions; tests/test_gpu_topology.py runs it on the
device and solves crowds whose topologies were only ever built there."""
import math

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import topology_selftest

EDGE = {
    "dropped_branch": ([-1, 0, 1, 1, 3, 0, 5, 6], [2, 7], [1, 2, 5, 6, 7], 2),
    "multi_root_released_origin": ([-1, 0, 1, -1, 3, 4], [2, 5], [1, 2, 4, 5], 1),
    "pinned_root": ([-1, 0, 1, 0, 3], [0, 2, 4], [1, 2, 3, 4], 2),
    "mid_chain_pin": ([-1, 0, 1, 2, 3, 4], [2, 5], [1, 2, 3, 4, 5], 2),
    "unsorted_parents": ([2, 2, -1, 1, 0], [3, 4], [0, 1, 3, 4], 2),
    "wide_fan_17_effectors": ([-1] + [0] * 17 + list(range(1, 18)), list(range(18, 35)), [], 0),
    "no_pins": ([-1, 0, 1], [], [], 0),
    "single_bone": ([-1], [0], [], 0),
    "three_roots": ([-1, 0, -1, 2, -1, 4, 5], [1, 6], [1, 3, 5, 6], 1),
}


def rig_of_workload(wl, **kw):
    t = wl.topo
    return (t.parents, wl.pins(), wl.constraints(), dict(iterations=t.iterations, max_cones=wl.cones.shape[2], **kw))


def rig(parents, pins, cons, ncones, **kw):
    pin_list = [dict(bone=b, weight=1.0) for b in pins]
    return (np.asarray(parents, np.int32), pin_list, [dict(bone=b, cone_count=ncones) for b in cons],
            dict(max_cones=max(1, ncones), **kw))


def random_rig(seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(1, 60))
    parents = [-1] + [int(rng.integers(-1 if rng.random() < 0.05 else 0, b)) for b in range(1, B)]
    if rng.random() < 0.3:                                   # unsorted: permute the bone indices
        perm = rng.permutation(B)
        inv = np.argsort(perm)
        parents = [int(inv[parents[perm[i]]]) if parents[perm[i]] >= 0 else -1 for i in range(B)]
    P = int(rng.integers(0, min(B, 12) + 1))
    pins = []
    for b in rng.choice(B, size=P, replace=bool(rng.random() < 0.2)):
        pr = [float(x) if rng.random() < 0.7 else 0.0 for x in rng.uniform(0, 1, 3)]
        pins.append(dict(bone=int(b), weight=float(rng.choice([0.0, 0.5, 1.0, 2.5])), direction_priorities=tuple(pr),
                         motion_propagation_factor=float(rng.choice([-0.5, 0.0, 0.3, 1.0, 1.7]))))
    mc = int(rng.integers(1, 4))
    cons = [dict(bone=int(b), cone_count=int(rng.integers(0, mc + 1))) for b in rng.choice(B, size=int(rng.integers(0, B + 1)))]
    kw = dict(max_cones=mc, iterations=int(rng.integers(0, 20)), default_damp=float(rng.uniform(0.01, 0.5)),
              stabilization_passes=int(rng.integers(0, 3)), constraint_mode=bool(rng.random() < 0.2))
    if rng.random() < 0.4:
        kw["bone_damp"] = rng.uniform(0.0, 0.6, int(rng.integers(1, B + 1))).astype(np.float32)
    return (np.asarray(parents, np.int32), pins, cons, kw)


def all_rigs():
    rigs = [rig_of_workload(W.generate(c, 1)) for c in (1, 2, 3, 4, 5)]
    rigs += [rig_of_workload(W.generate(2, 1), stabilization_passes=2), rig_of_workload(W.generate(5, 1), constraint_mode=True)]
    rigs += [rig(*v) for v in EDGE.values()]
    rigs += [random_rig(s) for s in range(200)]
    # refused descriptions: both builders must refuse them with the same message
    rigs += [rig([1, 0], [0], [], 0), rig([-1, 5], [0], [], 0), rig([-1, 0], [7], [], 0),
             rig([-1, 0, 1], [2], [9], 1), (np.asarray([-1, 0], np.int32), [dict(bone=1)], [dict(bone=1, cone_count=5)], dict(max_cones=2))]
    return rigs


def test_topo_builder_equals_host_builder():
    rigs = all_rigs()
    mism, err = topology_selftest(rigs, device=-1)
    bad = [i for i, m in enumerate(mism) if m]
    assert not bad, f"rigs {bad[:10]} differ: {err}"


def test_negative_bone_damp_count_is_refused_by_both_builders():
    """A negative bone_damp_count is refused with the same message by the host builder
    (mbik_plan_create / mbik_describe_topology) and the device-side one (build_topologies:
    mbik_plan_create_device would otherwise copy a reversed range)."""
    import ctypes as C
    from many_bone_ik_amd import _lib
    from many_bone_ik_amd.solver import _rig_arrays
    L = _lib.load()
    rigs = [rig([-1, 0, 1], [2], [], 0, bone_damp=np.full(3, 0.1, np.float32))] * 2
    descs, cfgs, keep = _rig_arrays(rigs)
    cfgs[1].bone_damp_count = -1
    assert L.mbik_describe_topology(C.byref(descs[1]), C.byref(cfgs[1]), None, None, None, None, None, None) == _lib.MBIK_EINVAL
    assert "negative count" in _lib.last_error()
    out = (C.c_int32 * 2)()
    assert L.mbik_selftest_topology(2, descs, cfgs, -1, out) == 0
    assert list(out) == [0, 0], _lib.last_error()
