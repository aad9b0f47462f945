"""The device's transcendental call sites against the host libm -- the reference's -- on every
float input (mbik_selftest_libm).  Godot's Math::sin/cos/acos(float) call ::sinf/::cosf/::acosf
and Math::sin/cos(double) call ::sin/::cos (glibc 2.35 on Linux x86-64); the product's
gd_math.h restates glibc's float algorithms for the device and uses the device's own double
sin/cos, so each call site is proven equal here:
  sin_f, cos_f, acos_f         all 2^32 float inputs
  slerp_scale0                 all 2^32 omega: (float)(sin((double)w) / (double)sinf(w)),
                               Quaternion::slerp's weight-0 coefficient (ik_bone_segment_3d.cpp:148-151);
                               its sinf is the branch-free glibc::sinf_small for |w| <= 1.6
  acosf_unit                   all 2^32 x: the slerp's acosf call site (branch-free for -0.5 < x < 1)
  cos((double)x)               all 2^32 float x: the cone radius cosines (setup)
  cos(x), x double             2^26 random tangent-radius-like doubles (setup; not enumerable)
The device's double cos (OCML) is not glibc's: it differs in the last bit on ~1.6 % of the
float inputs.  The setup only compares these cosines with float-valued doubles
(closest_to_cone, get_on_great_tangent_triangle) or rounds them to float, so the two COS
checks require observable equality (no float between the two results, same float rounding)
and report the raw bit differences; the solve's own call sites are bitwise.
Expected values come from oracle/libm_ref.c (platform libm), chunk by chunk."""
import os

import numpy as np
import pytest

from many_bone_ik_amd import _lib

pytestmark = pytest.mark.gpu

CHUNK = 1 << 26
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _check(mbik, oracle, fn, first, count, inputs=None, exp_fn=None):
    import ctypes
    import torch
    dev = torch.device("cuda", 0)
    exp = torch.from_numpy(oracle.libm_fill(fn if exp_fn is None else exp_fn, first, count, inputs, threads=THREADS)).to(dev)
    inp = torch.from_numpy(inputs).to(dev) if inputs is not None else None
    out = (ctypes.c_uint64 * 3)()
    rc = mbik.mbik_selftest_libm(fn, first, count, inp.data_ptr() if inp is not None else None, exp.data_ptr(), out,
                                 torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(rc)
    return int(out[0]), int(out[1]), int(out[2])


@pytest.mark.parametrize("fn,name", [(_lib.LIBM_SINF, "sinf"), (_lib.LIBM_COSF, "cosf"), (_lib.LIBM_ACOSF, "acosf"),
                                     (_lib.LIBM_SLERP_SCALE0, "slerp_scale0"),
                                     (_lib.LIBM_COS_F64_OF_F32, "cos_f64_of_f32"),
                                     (_lib.LIBM_ACOSF_UNIT, "acosf_unit")])
def test_all_float_inputs(mbik, oracle, fn, name):
    # acosf_unit: the slerp's branch-free acosf (gd_math.h glibc::acosf_unit), against the host acosf
    exp_fn = _lib.LIBM_ACOSF if fn == _lib.LIBM_ACOSF_UNIT else None
    bad_total, first_bad, bits = 0, None, 0
    for first in range(0, 1 << 32, CHUNK):
        bad, lo, diff = _check(mbik, oracle, fn, first, CHUNK, exp_fn=exp_fn)
        if bad and first_bad is None:
            first_bad = first + lo
        bad_total += bad
        bits += diff
    print(f"{name}: {bits} of 2^32 results differ in any bit, {bad_total} observably")
    if fn != _lib.LIBM_COS_F64_OF_F32:
        assert bits == 0
    assert bad_total == 0, (f"{name}: {bad_total} of 2^32 inputs differ from the host libm; first bit pattern "
                            f"{first_bad:#010x} ({np.uint32(first_bad).view(np.float32)!r})")


def test_cos_double_sample(mbik, oracle):
    """Tangent radii (pi - rA - rB) / 2 and the radii plus them: doubles in (0, pi]."""
    rng = np.random.default_rng(20240807)
    ra, rb = rng.uniform(1e-6, np.pi / 2, (2, CHUNK // 2))
    tr = (np.pi - (ra + rb)) / 2
    x = np.concatenate([tr, ra + tr])
    bad, lo, diff = _check(mbik, oracle, _lib.LIBM_COS_F64, 0, x.size, x)
    print(f"cos(double): {diff} of {x.size} results differ in any bit, {bad} observably")
    assert bad == 0, f"cos(double): {bad} of {x.size} differ; first input {x[lo]!r}"


def test_selftest_libm_rejects_bad_arguments(mbik):
    import ctypes
    out = (ctypes.c_uint64 * 3)()
    assert mbik.mbik_selftest_libm(10, 0, 1, None, None, out, None) == _lib.MBIK_EINVAL
    assert mbik.mbik_selftest_libm(_lib.LIBM_SINF, 1 << 32, 1, None, ctypes.c_void_p(8), out, None) == _lib.MBIK_EINVAL
    assert mbik.mbik_selftest_libm(_lib.LIBM_COS_F64, 0, 1, None, ctypes.c_void_p(8), out, None) == _lib.MBIK_EINVAL
