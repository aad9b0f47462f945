"""C ABI surface without a GPU: symbols, host-only topology query vs the oracle, error paths."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, describe_topology

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "mbik.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|void|const char \*)\s*(mbik_\w+)\(", src, re.M)))


def test_header_declares_and_library_exports_every_symbol(mbik):
    fns = header_functions()
    assert len(fns) >= 10
    assert set(fns) == set(_lib.EXPORTED_SYMBOLS)
    lib = C.CDLL(_lib.LIB_PATH)
    for f in fns:
        assert hasattr(lib, f), f


def _edge_topologies():
    # dropped (unpinned) branch, multi-root, pinned root, pin in mid-chain, deep single chain
    yield "dropped_branch", [-1, 0, 1, 1, 3, 0, 5], [2, 6], []
    yield "multi_root", [-1, 0, 1, -1, 3, 4], [2, 5], [1, 4]
    yield "pinned_root", [-1, 0, 1, 0, 3], [0, 2, 4], [1, 3]
    yield "mid_chain_pin", [-1, 0, 1, 2, 3, 4], [2, 5], [1, 2, 3, 4, 5]
    yield "unsorted_parents", [2, 2, -1, 1, 0], [3, 4], [0, 1]


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_describe_topology_matches_oracle(oracle, mbik, cfg):
    wl = W.generate(cfg, 1)
    o = oracle.Oracle(wl)
    d = describe_topology(wl.topo.parents, wl.pins())
    assert d["bone_list"].tolist() == o.bone_list()
    r, t, nh = o.segment_table()
    assert np.array_equal(d["seg_root"], r) and np.array_equal(d["seg_tip"], t) and np.array_equal(d["seg_headings"], nh)


@pytest.mark.parametrize("name,parents,pins,cons", list(_edge_topologies()), ids=[x[0] for x in _edge_topologies()])
def test_describe_edge_topologies_match_oracle(oracle, mbik, name, parents, pins, cons):
    topo = W.custom_topology(parents, pins, cons, cones_per_bone=1, twist=(0.1, 1.0))
    wl = W.generate(9, 1, topo=topo)
    o = oracle.Oracle(wl)
    d = describe_topology(parents, wl.pins())
    assert d["bone_list"].tolist() == o.bone_list()
    r, t, nh = o.segment_table()
    assert np.array_equal(d["seg_root"], r) and np.array_equal(d["seg_tip"], t) and np.array_equal(d["seg_headings"], nh)


def test_invalid_descriptions_are_rejected(mbik):
    with pytest.raises(_lib.MbikError) as e:
        describe_topology([0, 0], [dict(bone=1, weight=1)])  # cycle / self parent
    assert e.value.code == _lib.MBIK_EINVAL
    with pytest.raises(_lib.MbikError):
        describe_topology([-1, 0], [dict(bone=5, weight=1)])  # pin out of range
    with pytest.raises(_lib.MbikError):
        describe_topology([-1, 7], [])  # parent out of range


def test_plan_create_without_device_fails_loudly(mbik):
    from tests.conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is visible")
    wl = W.generate(3, 2)
    with pytest.raises(_lib.MbikError) as e:
        Plan.from_workload(wl)
    assert e.value.code == _lib.MBIK_ENODEV
