"""Child process of tests/test_gpu_libm_variant.py, started with GLIBC_TUNABLES set so that
THIS process's glibc picks the SSE2 build of sinf/cosf (and of sin/cos): the platform libm
is then the one a reference host without FMA would call.  Prints one JSON line.

    python tests/libm_variant_child.py selftest   # mbik_selftest_libm SSE2 codes, all 2^32 inputs
    python tests/libm_variant_child.py parity     # C1-C5 + discriminating rigs vs the oracle
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# inputs where glibc's FMA and SSE2 builds of sinf / cosf differ (tools/libm_exhaustive.c)
SIN_DISCRIMINATING = float.fromhex("0x1.ab6152p+5")
COS_DISCRIMINATING = float.fromhex("0x1.1475b6p+4")


def platform_is_sse2() -> bool:
    from oracle import pyoracle as po
    u = int(np.float32(SIN_DISCRIMINATING).view(np.uint32))
    n, _ = po.libm_restated_mismatches(0, u, 1, 1)  # restatement = the FMA build
    return n == 1


def selftest():
    import torch
    from many_bone_ik_amd import _lib
    from oracle import pyoracle as po
    mbik = _lib.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    chunk = 1 << 26
    res = {}
    for host_fn, dev_fn, name in ((_lib.LIBM_SINF, _lib.LIBM_SINF_SSE2, "sinf"), (_lib.LIBM_COSF, _lib.LIBM_COSF_SSE2, "cosf"),
                                  (_lib.LIBM_SLERP_SCALE0, _lib.LIBM_SLERP_SCALE0_SSE2, "slerp_scale0")):
        bad_total, bits, first_bad = 0, 0, None
        for first in range(0, 1 << 32, chunk):
            exp = torch.from_numpy(po.libm_fill(host_fn, first, chunk, None, threads=threads)).to(dev)
            out = (ctypes.c_uint64 * 3)()
            _lib.check(mbik.mbik_selftest_libm(dev_fn, first, chunk, None, exp.data_ptr(), out, st))
            if out[0] and first_bad is None:
                first_bad = first + int(out[1])
            bad_total += int(out[0])
            bits += int(out[2])
        res[name] = {"mismatches": bad_total, "bits_differ": bits, "first_bad": first_bad}
    return res


def discriminating(wl, which: str):
    """wl with every twist moved so the setup evaluates sinf / cosf at an input where the two
    glibc builds differ: set_axial_limits' axis-angle of min_angle (sinf(min_angle / 2),
    ik_kusudama_3d.cpp:103-115) or cos(range / 4) (:112)."""
    tw = wl.twist.copy()
    if which == "sin":
        tw[..., 0] = np.float32(2.0 * SIN_DISCRIMINATING)
    else:
        tw[..., 1] = np.float32(4.0 * COS_DISCRIMINATING)
    return dataclasses.replace(wl, twist=tw)


def parity():
    from many_bone_ik_amd import workloads as W
    from many_bone_ik_amd.solver import Plan
    from oracle import pyoracle as po
    out = {}
    cases = [(f"C{c}", W.generate(c, n, first=31)) for c, n in ((1, 1), (2, 24), (3, 24), (4, 8), (5, 4))]
    base = W.generate(2, 16, first=77)
    cases += [("C2_twist_sin", discriminating(base, "sin")), ("C2_twist_cos", discriminating(base, "cos"))]
    for name, wl in cases:
        ref = po.Oracle(wl).solve(wl.pose, wl.targets, threads=8)  # platform libm: the SSE2 build here
        r, tables = {}, []
        for v in (0, 1):
            p = Plan.from_workload(wl, libm_variant=v)
            got = p.solve_host(wl.pose, wl.targets)
            assert p.info()["libm_variant"] == v
            tables.append(p.setup_tables())
            p.close()
            r[f"variant{v}_bitwise"] = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
        r["tables_differ"] = any(not np.array_equal(a.view(np.uint8), b.view(np.uint8)) for a, b in zip(*tables))
        out[name] = r
    return out


if __name__ == "__main__":
    result = {"platform_sse2": platform_is_sse2()}
    result.update(selftest() if sys.argv[1] == "selftest" else parity())
    print(json.dumps(result), flush=True)
