"""The oracle against the reference's own known-answer tests (tests/golden/reference_kats.json,
re-expressed from tests/test_qcp.h, tests/test_ik_kusudama_3d.h, tests/test_ik_node_3d.h)."""
import json
import math
import os

import numpy as np
import pytest

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
EPS = KATS["epsilon"]


def qxform(q, v):
    u = np.array(q[:3], np.float64)
    uv = np.cross(u, v)
    return v + 2.0 * (uv * q[3] + np.cross(u, uv))


@pytest.mark.parametrize("case", KATS["qcp"], ids=lambda c: c["name"])
def test_qcp_kat(oracle, case):
    moved = np.array(case["moved"], np.float32)
    tr = np.array(case["translation"], np.float32)
    q = np.array(case["rotation"], np.float64)
    target = np.array([qxform(q, (m + tr).astype(np.float64)) for m in moved], np.float32)
    rot, trans = oracle.qcp(moved, target, np.array(case["weights"], np.float64), case["translate"], case["precision"])
    exp = np.array(case["expect_quat"])
    if case["expect"] == "equal":
        assert np.all(np.abs(rot - exp) < EPS), (rot, exp)
        if "expect_translation" in case:
            back = qxform(np.array([-q[0], -q[1], -q[2], q[3]]), trans.astype(np.float64))  # xform_inv
            assert np.all(np.abs(back - np.array(case["expect_translation"])) < EPS)
    else:  # tests/test_qcp.h:87-113: every component differs (degenerate collinear input -> identity)
        assert np.all(np.abs(rot - exp) > EPS), rot
        back = qxform(np.array([-q[0], -q[1], -q[2], q[3]]), trans.astype(np.float64))
        assert np.all(np.abs(back - np.array(case["expect_translation"])) > EPS)


@pytest.mark.parametrize("case", KATS["kusudama_point_in_limits"], ids=lambda c: c["name"])
def test_point_in_limits_kat(oracle, case):
    cones = np.array(case["cones"], np.float32)
    cones[:, 3] = np.float32(case["cones"][0][3])
    out, ib = oracle.local_point_in_limits(cones, np.array(case["point"], np.float32), np.array(case["tangents"]))
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


@pytest.mark.parametrize("case", KATS["closest_path_point"], ids=lambda c: c["name"])
def test_closest_path_point_kat(oracle, case):
    use_next = {"null": 0, "self": 1, "next": 2}[case["next"]]
    out = oracle.closest_path_point(np.array(case["cones"], np.float32), case["cone"], use_next,
                                    np.array(case["point"], np.float32), np.array(case["tangents"], np.float32))
    assert np.array_equal(out, np.array(case["expect_point"], np.float32))


@pytest.mark.parametrize("case", KATS["ik_node"], ids=lambda c: c["name"])
def test_ik_node_kat(oracle, case):
    if case["op"] == "affine_inverse_roundtrip":
        x = np.array(case["xform"], np.float32)
        back = oracle.xform_affine_inverse(oracle.xform_affine_inverse(x))
        assert np.array_equal(back, x)
    elif case["op"] == "to_local_global":
        x = np.array(case["xform"], np.float32)
        p = np.array(case["point"], np.float32)
        inv = oracle.xform_affine_inverse(x)
        local = inv[:9].reshape(3, 3) @ p + inv[9:]
        glob = x[:9].reshape(3, 3) @ local + x[9:]
        assert np.array_equal(glob.astype(np.float32), p)
    else:  # local = parent_global.affine_inverse() * global
        pg = np.array(case["parent_global"], np.float32)
        cg = np.array(case["child_global"], np.float32)
        local = oracle.xform_mul(oracle.xform_affine_inverse(pg), cg)
        assert np.array_equal(local, np.array(case["expect_local"], np.float32))


def test_cone_tangent_circles_are_unit_and_outside_cones(oracle):
    """update_tangent_handles (ik_open_cone_3d.cpp:36-120): tangent centres on the unit sphere,
    tangent radius (pi - rA - rB) / 2, each circle touching both cones."""
    ra, rb = math.radians(35), math.radians(20)
    a = np.array([0, 1, 0], np.float32)
    b = np.array([math.sin(math.radians(60)), math.cos(math.radians(60)), 0], np.float32)
    tg = oracle.cone_tangents(np.array([[*a, ra], [*b, rb]], np.float32))
    t1, t2, tr = tg[0, 0:3], tg[0, 3:6], tg[0, 6]
    assert abs(np.linalg.norm(t1) - 1) < 1e-6 and abs(np.linalg.norm(t2) - 1) < 1e-6
    assert abs(tr - (math.pi - ra - rb) / 2) < 1e-6
    for t in (t1, t2):
        assert abs(math.acos(np.clip(t @ a, -1, 1)) - (ra + tr)) < 1e-3
        assert abs(math.acos(np.clip(t @ b, -1, 1)) - (rb + tr)) < 1e-3
