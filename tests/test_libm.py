"""The reference's libm (CPU): Godot's Math::sin/cos/acos(float) call ::sinf/::cosf/::acosf,
glibc on Linux x86-64.  The oracle calls the platform libm; oracle/glibc_libm.h restates
glibc 2.35's algorithms (the product's gd_math.h restates them independently for the
device).  These tests pin which glibc build the host runs: the restatement must match the
platform on a strided sweep of all float inputs, and on the inputs where glibc's FMA and
SSE2 ifunc variants differ (tools/libm_exhaustive.c, profiles/r02_libm_exhaustive.txt:
0 mismatches for the FMA variant over all 2^32 inputs)."""
import numpy as np
import pytest

# inputs where the SSE2 build of sinf/cosf differs from the FMA build (the first of the 12 /
# 22 tools/libm_exhaustive.c lists): the platform must agree with the FMA build on them
FMA_DISCRIMINATING = {0: ["0x1.ab6152p+5", "0x1.46b80ep+6", "0x1.46ba88p+6", "0x1.52e6cp+6"],
                      1: ["0x1.1475b6p+4", "0x1.1475b8p+4", "0x1.1475bap+4", "0x1.1475bcp+4"]}


@pytest.mark.parametrize("fn,name", [(0, "sinf"), (1, "cosf"), (2, "acosf")])
def test_restated_glibc_matches_platform_sweep(oracle, fn, name):
    # every 4099th bit pattern (~1.05 M inputs over all signs, exponents, NaN/inf) plus a
    # dense run over [0.5, 2) where the solve's angles live
    n, bad = oracle.libm_restated_mismatches(fn, 0, (1 << 32) // 4099, 4099)
    assert n == 0, f"{name}: {n} mismatches, first bit pattern {bad:#x}"
    lo = int(np.float32(0.5).view(np.uint32))
    n, bad = oracle.libm_restated_mismatches(fn, lo, 1 << 22, 3)
    assert n == 0, f"{name}: {n} mismatches in [0.5, 2), first {bad:#x}"


@pytest.mark.parametrize("fn", [0, 1])
def test_platform_is_fma_variant(oracle, fn):
    for x in FMA_DISCRIMINATING[fn]:
        u = int(np.float32(float.fromhex(x)).view(np.uint32))
        n, _ = oracle.libm_restated_mismatches(fn, u, 1, 1)
        assert n == 0, f"platform libm disagrees with the FMA build at {x!r}: not glibc 2.35's FMA sinf/cosf"


def test_libm_fill_matches_restatement(oracle):
    """libm_fill (the GPU self-test's expected values) agrees with the restatement."""
    v = oracle.libm_fill(0, int(np.float32(0.25).view(np.uint32)), 1 << 16)
    assert v.dtype == np.float32 and np.isfinite(v).all()
    n, _ = oracle.libm_restated_mismatches(0, int(np.float32(0.25).view(np.uint32)), 1 << 16, 1)
    assert n == 0
