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


def _gdmath_checker():
    """tools/gdmath_host_check.cpp: the product's own gd_math.h (host build) vs the platform libm."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "gdmath_host_check_test")
    src = os.path.join(root, "tools", "gdmath_host_check.cpp")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(
            os.path.join(root, "many_bone_ik_amd", "csrc", "gd_math.h"))):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", "-pthread", "-I",
                        os.path.join(root, "many_bone_ik_amd", "csrc"), src, "-o", exe], check=True)
    return exe


def _run_checker(variant, sse2_platform, *args):
    import os
    import re
    import subprocess
    from many_bone_ik_amd import _lib
    env = dict(os.environ)
    env.pop("GLIBC_TUNABLES", None)
    if sse2_platform:
        env["GLIBC_TUNABLES"] = _lib.GLIBC_SSE2_TUNABLES
    out = subprocess.run([_gdmath_checker(), str(variant), *args], capture_output=True, text=True, env=env,
                         check=True).stdout
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"^(\w+)\s+variant \w+ mismatches .*?: (\d+)", out, re.M)}


@pytest.mark.parametrize("variant,sse2_platform", [(0, False), (1, True)])
def test_product_libm_variants_match_their_glibc_build(variant, sse2_platform):
    """gd_math.h's sinf/cosf (the kernel's source, host build) in each libm_variant equal the
    platform glibc built the same way -- the FMA build by default, the SSE2 build when
    GLIBC_TUNABLES disables the FMA ifunc -- on a strided sweep and on the discriminating
    inputs; the other pairing differs on those inputs (so the tunable really switches)."""
    disc = FMA_DISCRIMINATING[0] + FMA_DISCRIMINATING[1]
    assert all(v == 0 for v in _run_checker(variant, sse2_platform, "4099").values())
    assert all(v == 0 for v in _run_checker(variant, sse2_platform, "list", *disc).values())
    crossed = _run_checker(1 - variant, sse2_platform, "list", *disc)
    assert crossed["sin_f"] == 4 and crossed["cos_f"] == 4 and crossed["acos_f"] == 0


def test_branch_free_slerp_forms_match_glibc_restatements():
    """tools/branchfree_check.cpp: gd_math.h's branch-free sinf (|y| <= 1.6) and acosf
    (-0.5 < x < 1), used by the solve's slerp coefficient, against the branchy restatements on
    every 97th float of their ranges (the full ranges and the device: tests/test_gpu_libm.py)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "branchfree_check_test")
    src = os.path.join(root, "tools", "branchfree_check.cpp")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", "-pthread", "-I",
                    os.path.join(root, "many_bone_ik_amd", "csrc"), src, "-o", exe], check=True)
    out = subprocess.run([exe, "97"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "FMA mismatches 0, SSE2 mismatches 0; acosf_unit mismatches 0" in out.stdout
