"""The kernel's float quotients against IEEE division on the device (mbik_selftest_div).

The reference divides in float (x86 divss, Godot real_t); the solve computes those quotients
through an fp64 reciprocal (gd_math.h: gd_quot with one residual correction, gd_pow2_over
for the power-of-two numerators of Basis::set_quaternion / get_quaternion / inverse, and
gd_sqrt_rcp for normalized()'s reciprocal of the rounded length).  Each must round exactly as
IEEE division does; the self-test enumerates:
  every pair of 24 special operands; all 2^32 dividends for 12 divisors; 0.5 / b, 1 / b and
  2 / b for all 2^32 divisors; a / sqrtf(l) and sqrtf(l) for all 2^32 l and 8 dividends;
  2^31 random pairs; 2^31 constructed denormal midpoint quotients (the one case where a
  quotient of two floats can be a rounding midpoint).
"""
import ctypes

import pytest

from many_bone_ik_amd import _lib

pytestmark = pytest.mark.gpu

CLASSES = ["specials", "all_dividends", "random", "midpoints", "pow2_numerator", "normalize"]


def test_quotients_equal_ieee_division(mbik):
    out = (ctypes.c_uint64 * 20)()
    _lib.check(mbik.mbik_selftest_div(0, 1024, out))
    counts = dict(zip(CLASSES, [int(out[i]) for i in range(len(CLASSES))]))
    print("division self-test mismatches:", counts)
    bad = {c: (hex(out[8 + 2 * i]), hex(out[9 + 2 * i])) for i, c in enumerate(CLASSES) if out[i]}
    assert not any(counts.values()), f"mismatching quotients {counts}, first operands {bad}"


def test_selftest_div_rejects_bad_arguments(mbik):
    out = (ctypes.c_uint64 * 20)()
    assert mbik.mbik_selftest_div(0, 0, None) == _lib.MBIK_EINVAL
    assert mbik.mbik_selftest_div(999, 0, out) == _lib.MBIK_EINVAL
