"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the plan
builder -- ManyBoneIK3D::_bone_list_changed's segmentation and heading weights
(plan.cpp build_topology), the per-skeleton setup on host threads (build_skeletons / setup.h)
and every launch schedule build_schedule can produce -- and the oracle (object graph, one frame
on 1 and 3 threads), on C1-C5 and the edge topologies of the GPU edge-case tests.  The
drivers and their Makefile are in tools/san/; they build with g++/gcc (no GPU needed)."""
import fcntl
import math
import os
import struct
import subprocess

import numpy as np
import pytest

from many_bone_ik_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "san")

EDGE = {
    "dropped_branch": ([-1, 0, 1, 1, 3, 0, 5, 6], [2, 7], [1, 2, 5, 6, 7], 2, (0.2, 1.5)),
    "multi_root_released_origin": ([-1, 0, 1, -1, 3, 4], [2, 5], [1, 2, 4, 5], 1, (-0.3, 2.0)),
    "pinned_root": ([-1, 0, 1, 0, 3], [0, 2, 4], [1, 2, 3, 4], 2, (0.0, math.tau)),
    "unsorted_parents": ([2, 2, -1, 1, 0], [3, 4], [0, 1, 3, 4], 2, (0.0, 1.0)),
    "three_cones": ([-1, 0, 1, 2, 0, 4, 5], [3, 6], [1, 2, 3, 4, 5, 6], 3, (0.0, 1.0)),
    "zero_cones": ([-1, 0, 1, 2, 0, 4, 5], [3, 6], [1, 2, 3, 4, 5, 6], 0, (0.0, 0.3)),
    "wide_fan_17_effectors": ([-1] + [0] * 17 + list(range(1, 18)), list(range(18, 35)), [], 0, None),
    "no_pins": ([-1, 0, 1], [], [], 0, None),
    "single_bone": ([-1], [0], [], 0, None),
}


def write_case(path, wl, constraint_mode=0, stab=0):
    t = wl.topo
    B, P, C = wl.bone_count, int(t.pins.shape[0]), int(t.constrained.shape[0])
    mc = int(wl.cones.shape[2])
    bd = np.zeros(0, np.float32) if wl.bone_damp is None else np.asarray(wl.bone_damp, np.float32)
    with open(path, "wb") as f:
        f.write(b"MBKC")
        f.write(struct.pack("<9i", B, P, C, mc, t.iterations, wl.n, constraint_mode, stab, bd.shape[0]))
        f.write(struct.pack("<f", wl.default_damp))
        for a, dt in ((t.parents, np.int32), (t.pins, np.int32), (wl.pin_weight, np.float32),
                      (wl.pin_priority, np.float32), (wl.pin_propagation, np.float32), (t.constrained, np.int32),
                      (wl.cone_count, np.int32), (bd, np.float32), (wl.pose, np.float32), (wl.targets, np.float32),
                      (wl.cones, np.float32), (wl.twist, np.float32)):
            f.write(np.ascontiguousarray(a, dt).tobytes())


@pytest.fixture(scope="module")
def drivers():
    # one make at a time: pytest-xdist workers each run this fixture, and a worker executing a
    # driver while another relinks it fails with a PermissionError
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "san")], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stderr[-3000:])
    return os.path.join(OUT, "plan_san"), os.path.join(OUT, "oracle_san")


def _cases():
    out = [(f"c{cfg}", lambda cfg=cfg, n=n: W.generate(cfg, n), {}) for cfg, n in ((1, 1), (2, 3), (3, 3), (4, 2), (5, 1))]
    out.append(("c2_stab2", lambda: W.generate(2, 2), {"stab": 2}))
    out.append(("c2_constraint_mode", lambda: W.generate(2, 2), {"constraint_mode": 1}))
    for name, (parents, pins, cons, nc, twist) in EDGE.items():
        out.append((name, lambda p=parents, q=pins, c=cons, k=nc, t=twist:
                    W.generate(11, 2, topo=W.custom_topology(p, q, c, cones_per_bone=k, twist=t)), {}))
    return out


CASES = _cases()


@pytest.mark.parametrize("name,make,kw", CASES, ids=[c[0] for c in CASES])
def test_host_code_is_sanitizer_clean(drivers, tmp_path, name, make, kw):
    path = str(tmp_path / f"{name}.case")
    write_case(path, make(), **kw)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    # under tools/san/cpu_suite_asan.sh this process has clang's ASan runtime preloaded; the
    # gcc-built drivers bring their own, so only that entry is dropped for them
    pre = [x for x in env.get("LD_PRELOAD", "").split() if "libclang_rt.asan" not in x]
    if "LD_PRELOAD" in env:
        env["LD_PRELOAD"] = " ".join(pre)
    for exe in drivers:
        r = subprocess.run([exe, path], capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0, f"{os.path.basename(exe)} {name}:\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
        assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
        assert r.stdout.startswith(("ok", "build_topology refused", "build_skeletons refused", "oracle_create refused"))
