"""The plan's libm_variant (mbik_plan_options, include/mbik.h): which glibc build of sinf/cosf
the reference host runs.  A reference on a CPU without FMA -- or with glibc's FMA ifunc
disabled (GLIBC_TUNABLES=glibc.cpu.hwcaps=-FMA,-AVX2_Usable) -- calls the SSE2 build, which
differs from the FMA build on 12 (sinf) and 22 (cosf) of the 2^32 float inputs.  Each check
runs in a child process whose own glibc is switched to the SSE2 build (tests/libm_variant_child.py):
  * the device's SSE2 sinf, cosf and slerp coefficient equal that platform libm on all 2^32
    inputs (mbik_selftest_libm, codes *_SSE2);
  * plans created with libm_variant = SSE2 are bitwise equal to the oracle running on that
    libm for C1-C5 and for two rigs whose twist limits make the setup evaluate sinf / cosf
    at an input where the builds differ; those two build different setup tables under the two
    variants, and the default (FMA) plan's solve of the sinf one differs from that reference.
Needs an MI355X: -m gpu."""
import json
import os
import subprocess
import sys

import pytest

from many_bone_ik_amd import _lib

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(mode, timeout):
    env = dict(os.environ)
    env["GLIBC_TUNABLES"] = _lib.GLIBC_SSE2_TUNABLES
    r = subprocess.run([sys.executable, os.path.join(HERE, "libm_variant_child.py"), mode], capture_output=True, text=True,
                       env=env, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res.pop("platform_sse2"), "GLIBC_TUNABLES did not switch the child's libm to the SSE2 build"
    return res


def test_sse2_variant_all_float_inputs(oracle, mbik):
    res = _child("selftest", 240)
    print(res)
    for name, r in res.items():
        assert r["bits_differ"] == 0 and r["mismatches"] == 0, (name, r)


def test_sse2_variant_solves_bitwise(oracle, mbik):
    res = _child("parity", 240)
    print(res)
    for name, r in res.items():
        assert r["variant1_bitwise"], f"{name}: SSE2-variant plan differs from the oracle on an SSE2 libm"
        if name.startswith("C2_twist"):
            # the variant reaches the setup tables (the twist frame / half-cosine)...
            assert r["tables_differ"], f"{name}: both variants built the same setup tables"
        else:
            # ...while realistic angles (|x| < 17) never reach an input where the builds differ
            assert r["variant0_bitwise"] and not r["tables_differ"], f"{name}: variants differ on a realistic rig"
    # and the solve: the FMA plan of the sinf-discriminating rig differs from the SSE2 reference
    assert not res["C2_twist_sin"]["variant0_bitwise"]
