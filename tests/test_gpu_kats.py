"""The HIP device code against the reference's own known-answer tests.

tests/golden/reference_kats.json re-expresses the reference's unit tests as data
(tests/test_qcp.h:40-113, tests/test_ik_kusudama_3d.h:38-156, tests/test_ik_node_3d.h:39-106).
tests/test_oracle_kats.py pins the CPU oracle to them; here the solve kernel's own device
functions run on the same inputs (mbik_selftest_qcp / _point_in_limits / _xform, ABI 8): QCP's
weighted superpose through the one-lane heading branch's primitives and qcp_adjugate /
qcp_single, local_point_in_limits on a plan's setup tables, and the Transform3D product and
affine inverse.  Each result must meet the KAT's expectation within CMP_EPSILON and equal the
oracle bit for bit; so must both normalization forms of the kernel builds.  The KAT family
get_closest_path_point (test_ik_kusudama_3d.h:158-202) has no device counterpart: it serves
IKKusudama3D::local_point_on_path_sequence (ik_kusudama_3d.cpp:235-258), which the solve never
calls.  Needs an MI355X: -m gpu."""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd.solver import Plan

from .test_oracle_kats import qxform

pytestmark = pytest.mark.gpu

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
EPS = KATS["epsilon"]
FP = C.POINTER(C.c_float)


def _f(a):
    return np.ascontiguousarray(a, np.float32)


def dev_qcp(moved, target, weights, translate, precision):
    L = _lib.load()
    m, t, w = _f(moved).reshape(-1), _f(target).reshape(-1), np.ascontiguousarray(weights, np.float64)
    out = np.zeros(14, np.float32)
    _lib.check(L.mbik_selftest_qcp(w.shape[0], m.ctypes.data_as(FP), t.ctypes.data_as(FP),
                                   w.ctypes.data_as(C.POINTER(C.c_double)), int(translate), float(precision), 0,
                                   out.ctypes.data_as(FP)))
    assert np.array_equal(out[:7].view(np.uint32), out[7:].view(np.uint32)), "plain and select-form builds differ"
    return out[:4], out[4:7]


def dev_xform(op, a, b=None):
    L = _lib.load()
    a = _f(a)
    b = _f(a if b is None else b)
    out = np.zeros(12, np.float32)
    _lib.check(L.mbik_selftest_xform(op, a.ctypes.data_as(FP), b.ctypes.data_as(FP), 0, out.ctypes.data_as(FP)))
    return out


def kusudama_plan(cones):
    """A two-bone rig whose child carries one constraint with the KAT's cones: the plan's setup
    tables are then the reference's IKKusudama3D for them (constraint slot 0, skeleton 0)."""
    cones = _f(cones)
    n = cones.shape[0]
    pose = np.zeros((1, 2, 10), np.float32)
    pose[0, :, 3] = 1.0
    pose[0, :, 7:10] = 1.0
    pose[0, 1, 5] = 1.0
    pins = [dict(bone=1, weight=1.0, direction_priorities=(0.2, 0.0, 0.2), motion_propagation_factor=1.0)]
    return Plan([-1, 0], pins, [dict(bone=1, cone_count=n)], pose, cones.reshape(1, 1, n, 4),
                np.array([[[0.0, 2 * math.pi]]], np.float32), max_cones=n)


def dev_point_in_limits(plan, point):
    L = _lib.load()
    out = np.zeros(6, np.float32)
    ib = np.zeros(2, np.float64)
    _lib.check(L.mbik_selftest_point_in_limits(plan.h, 0, 0, _f(point).ctypes.data_as(FP), out.ctypes.data_as(FP),
                                               ib.ctypes.data_as(C.POINTER(C.c_double))))
    assert np.array_equal(out[:3].view(np.uint32), out[3:].view(np.uint32)) and ib[0] == ib[1]
    return out[:3], ib[0]


@pytest.mark.parametrize("case", KATS["qcp"], ids=lambda c: c["name"])
def test_device_qcp_kat(oracle, mbik, case):
    moved = np.array(case["moved"], np.float32)
    tr = np.array(case["translation"], np.float32)
    q = np.array(case["rotation"], np.float64)
    target = np.array([qxform(q, (m + tr).astype(np.float64)) for m in moved], np.float32)
    w = np.array(case["weights"], np.float64)
    rot, trans = dev_qcp(moved, target, w, case["translate"], case["precision"])
    o_rot, o_trans = oracle.qcp(moved, target, w, case["translate"], case["precision"])
    assert np.array_equal(rot.view(np.uint32), o_rot.view(np.uint32)), (rot, o_rot)
    assert np.array_equal(trans.view(np.uint32), o_trans.view(np.uint32)), (trans, o_trans)
    exp = np.array(case["expect_quat"])
    back = qxform(np.array([-q[0], -q[1], -q[2], q[3]]), trans.astype(np.float64))  # xform_inv
    if case["expect"] == "equal":
        assert np.all(np.abs(rot - exp) < EPS), (rot, exp)
        if "expect_translation" in case:
            assert np.all(np.abs(back - np.array(case["expect_translation"])) < EPS)
    else:  # tests/test_qcp.h:87-113: collinear input -> identity, every component differs
        assert np.all(np.abs(rot - exp) > EPS), rot
        assert np.all(np.abs(back - np.array(case["expect_translation"])) > EPS)


def _random_qcp_cases():
    rng = np.random.default_rng(20240807)
    cases = []
    for h in (1, 5, 20, 40, 80):
        for translate in (False, True):
            m = rng.normal(size=(h, 3)).astype(np.float32)
            ax = rng.normal(size=3)
            ax /= np.linalg.norm(ax)
            ang = rng.uniform(0, math.pi)
            q = np.array([*(ax * math.sin(ang / 2)), math.cos(ang / 2)])
            t = np.array([qxform(q, v.astype(np.float64)) for v in m], np.float32) + rng.normal(scale=0.01, size=(h, 3)).astype(np.float32)
            w = rng.choice([0.0, 0.25, 1.0, 2.0], h)
            w[0] = 1.0
            cases.append((f"H{h}_t{int(translate)}", m, t, w, translate))
    # degenerate inputs: collinear points, near-180-degree turns, a single antiparallel pair, zeros
    line = np.outer(np.arange(1, 6), [1, 2, 3]).astype(np.float32)
    cases.append(("collinear", line, line[::-1].copy(), np.ones(5), True))
    flip = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0]], np.float32)
    cases.append(("near_180", flip, (-flip + np.float32(1e-4)).astype(np.float32), np.ones(4), False))
    cases.append(("antiparallel_pair", np.array([[1, 2, 3]], np.float32), np.array([[-1, -2, -3]], np.float32), np.ones(1), False))
    cases.append(("zero_weights", flip, flip[::-1].copy(), np.zeros(4), True))
    cases.append(("zero_vectors", np.zeros((3, 3), np.float32), np.zeros((3, 3), np.float32), np.ones(3), False))
    return cases


@pytest.mark.parametrize("case", _random_qcp_cases(), ids=lambda c: c[0])
def test_device_qcp_matches_oracle(oracle, mbik, case):
    """SURVEY §8(c) golden-vector class (2): random QCP cases, H in {1, 5, 20, 40, 80}, translate
    on and off, and the degenerate inputs -- the device's QCP bitwise equal to the oracle's."""
    _, m, t, w, translate = case
    rot, trans = dev_qcp(m, t, w, translate, 1e-6)
    o_rot, o_trans = oracle.qcp(m, t, w, translate, 1e-6)
    assert np.array_equal(rot.view(np.uint32), o_rot.view(np.uint32)), (rot, o_rot)
    assert np.array_equal(trans.view(np.uint32), o_trans.view(np.uint32)), (trans, o_trans)


@pytest.mark.parametrize("case", KATS["kusudama_point_in_limits"], ids=lambda c: c["name"])
def test_device_point_in_limits_kat(oracle, mbik, case):
    cones = np.array(case["cones"], np.float32)
    point = np.array(case["point"], np.float32)
    out, ib = dev_point_in_limits(kusudama_plan(cones), point)
    o_out, o_ib = oracle.local_point_in_limits(cones, point, np.array(case["tangents"]))
    assert np.array_equal(out.view(np.uint32), o_out.view(np.uint32)) and ib == o_ib, (out, ib, o_out, o_ib)
    e = case["expect_in_bounds"]
    if e == "positive":
        assert ib > 0
    elif e == "negative":
        assert ib < 0
    else:
        assert ib == e
    exp = np.array(case["expect_point"], np.float32)
    if case["compare"] == "exact":
        assert np.array_equal(out, exp)
    else:  # Vector3::is_equal_approx
        tol = np.maximum(EPS * np.abs(out), EPS)
        assert np.all((out == exp) | (np.abs(out - exp) < tol)), (out, exp)


def test_device_point_in_limits_two_cones_matches_oracle(oracle, mbik):
    """Two cones with their tangent circles (the C2/C5 constraint shape): points inside either
    cone, in each tangent triangle and outside everything, bitwise against the oracle."""
    cones = np.array([[0, 1, 0, math.radians(35)], [math.sin(math.radians(45)), math.cos(math.radians(45)), 0,
                                                        math.radians(20)]], np.float32)
    plan = kusudama_plan(cones)
    rng = np.random.default_rng(7)
    for p in list(rng.normal(size=(64, 3)).astype(np.float32)) + [np.array([0, 0, 1], np.float32), np.array([0, -1, 0], np.float32)]:
        out, ib = dev_point_in_limits(plan, p)
        o_out, o_ib = oracle.local_point_in_limits(cones, p)
        assert np.array_equal(out.view(np.uint32), o_out.view(np.uint32)) and ib == o_ib, (p, out, ib, o_out, o_ib)


@pytest.mark.parametrize("case", KATS["ik_node"], ids=lambda c: c["name"])
def test_device_ik_node_kat(oracle, mbik, case):
    if case["op"] == "affine_inverse_roundtrip":
        x = np.array(case["xform"], np.float32)
        inv = dev_xform(1, x)
        assert np.array_equal(inv, oracle.xform_affine_inverse(x))
        assert np.array_equal(dev_xform(1, inv), x)
    elif case["op"] == "to_local_global":
        x = np.array(case["xform"], np.float32)
        p = np.array(case["point"], np.float32)
        inv = dev_xform(1, x)
        assert np.array_equal(inv, oracle.xform_affine_inverse(x))
        local = inv[:9].reshape(3, 3) @ p + inv[9:]
        glob = x[:9].reshape(3, 3) @ local + x[9:]
        assert np.array_equal(glob.astype(np.float32), p)
    else:  # local = parent_global.affine_inverse() * global
        pg = np.array(case["parent_global"], np.float32)
        cg = np.array(case["child_global"], np.float32)
        local = dev_xform(0, dev_xform(1, pg), cg)
        assert np.array_equal(local, oracle.xform_mul(oracle.xform_affine_inverse(pg), cg))
        assert np.array_equal(local, np.array(case["expect_local"], np.float32))


def test_device_xform_matches_oracle(oracle, mbik):
    rng = np.random.default_rng(11)
    for _ in range(64):
        a = rng.normal(size=12).astype(np.float32)
        b = rng.normal(size=12).astype(np.float32)
        assert np.array_equal(dev_xform(0, a, b).view(np.uint32), oracle.xform_mul(a, b).view(np.uint32))
        assert np.array_equal(dev_xform(1, a).view(np.uint32), oracle.xform_affine_inverse(a).view(np.uint32))


def test_kat_argument_checks(mbik):
    L = _lib.load()
    out = np.zeros(14, np.float32)
    z = np.zeros(3, np.float32)
    assert L.mbik_selftest_qcp(0, z.ctypes.data_as(FP), z.ctypes.data_as(FP), None, 0, 1e-6, 0, out.ctypes.data_as(FP)) == _lib.MBIK_EINVAL
    assert L.mbik_selftest_xform(2, z.ctypes.data_as(FP), z.ctypes.data_as(FP), 0, out.ctypes.data_as(FP)) == _lib.MBIK_EINVAL
