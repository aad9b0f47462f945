"""ctypes bindings for the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product (many_bone_ik_amd) never does.  See mbik_oracle.h for layouts and
ik_oracle.c for the reference file:line each restated function follows.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")  # override: libm study only
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


class OracleDesc(C.Structure):
    _fields_ = [
        ("bone_count", C.c_int32), ("parents", C.c_void_p),
        ("pin_count", C.c_int32), ("pin_bone", C.c_void_p), ("pin_weight", C.c_void_p),
        ("pin_priority", C.c_void_p), ("pin_propagation", C.c_void_p),
        ("constraint_count", C.c_int32), ("constraint_bone", C.c_void_p),
        ("constraint_cone_count", C.c_void_p), ("max_cones", C.c_int32),
        ("iterations", C.c_int32), ("default_damp", C.c_float), ("constraint_mode", C.c_int32),
        ("stabilization_passes", C.c_int32), ("bone_damp_count", C.c_int32), ("bone_damp", C.c_void_p),
    ]


def build() -> str:
    """Compile liboracle.so (gcc, seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE, "CC=gcc"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(OracleDesc), C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_solve.restype = C.c_int32
        L.oracle_solve.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_segment_count.argtypes = [C.c_void_p]
        L.oracle_segment_count.restype = C.c_int32
        L.oracle_bone_list.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_bone_list.restype = C.c_int32
        L.oracle_segment_table.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_segment_table.restype = C.c_int32
        L.oracle_segment_solve.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.oracle_segment_solve.restype = C.c_int32
        L.oracle_qcp.argtypes = [_f32p, _f32p, _f64p, C.c_int32, C.c_int32, C.c_double, _f32p, _f32p]
        L.oracle_local_point_in_limits.restype = C.c_double
        L.oracle_local_point_in_limits.argtypes = [_f32p, C.c_int32, C.c_void_p, _f32p, _f32p]
        L.oracle_closest_path_point.argtypes = [_f32p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32, _f32p, _f32p]
        L.oracle_cone_tangents.argtypes = [_f32p, C.c_int32, _f32p]
        L.oracle_xform_mul.argtypes = [_f32p, _f32p, _f32p]
        L.oracle_xform_affine_inverse.argtypes = [_f32p, _f32p]
        L.oracle_basis_to_quat.argtypes = [_f32p, _f32p]
        L.oracle_quat_to_basis.argtypes = [_f32p, _f32p]
        L.oracle_libm_fill.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_libm_fill.restype = C.c_int32
        L.oracle_libm_restated_mismatches.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.c_uint64,
                                                      C.POINTER(C.c_uint64)]
        L.oracle_libm_restated_mismatches.restype = C.c_uint64
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


class Oracle:
    """One reference object graph per skeleton of a workload (== _bone_list_changed)."""

    def __init__(self, wl, setup_pose=None, iterations=None, constraint_mode=False,
                 stabilization_passes=0, bone_damp=None, default_damp=None):
        L = lib()
        t = wl.topo
        self._keep = []

        def keep(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            self._keep.append(a)
            return a

        P = t.pins.shape[0]
        Cn = t.constrained.shape[0]
        d = OracleDesc()
        d.bone_count = t.parents.shape[0]
        d.parents = _ptr(keep(t.parents, np.int32))
        d.pin_count = P
        d.pin_bone = _ptr(keep(t.pins, np.int32))
        d.pin_weight = _ptr(keep(np.broadcast_to(np.asarray(wl.pin_weight, np.float32), (P,)), np.float32))
        d.pin_priority = _ptr(keep(np.broadcast_to(np.asarray(wl.pin_priority, np.float32), (P, 3)), np.float32))
        d.pin_propagation = _ptr(keep(np.broadcast_to(np.asarray(wl.pin_propagation, np.float32), (P,)), np.float32))
        d.constraint_count = Cn
        d.constraint_bone = _ptr(keep(t.constrained, np.int32))
        cc = getattr(wl, "cone_count", None)
        d.constraint_cone_count = _ptr(keep(np.full(Cn, t.cones_per_bone) if cc is None else cc, np.int32))
        d.max_cones = wl.cones.shape[2]
        d.iterations = t.iterations if iterations is None else iterations
        d.default_damp = wl.default_damp if default_damp is None else default_damp
        d.constraint_mode = int(constraint_mode)
        d.stabilization_passes = stabilization_passes
        if bone_damp is None:
            bone_damp = getattr(wl, "bone_damp", None)
        bd = keep(np.zeros(0) if bone_damp is None else bone_damp, np.float32)
        d.bone_damp_count = bd.shape[0]
        d.bone_damp = _ptr(bd) if bd.shape[0] else None
        self.desc = d
        self.n = wl.n
        self.B = d.bone_count
        self.P = P
        self.iterations = d.iterations
        sp = keep(wl.pose if setup_pose is None else setup_pose, np.float32)
        cones = keep(wl.cones, np.float32)
        twist = keep(wl.twist, np.float32)
        self.h = L.oracle_create(C.byref(d), wl.n, _ptr(sp), _ptr(cones), _ptr(twist))

    def solve(self, pose_in, targets, first=0, count=None, threads=1, trace=False):
        L = lib()
        count = self.n - first if count is None else count
        pose_in = np.ascontiguousarray(pose_in, np.float32)
        targets = np.ascontiguousarray(targets, np.float32)
        assert pose_in.shape == (count, self.B, 10) and targets.shape == (count, self.P, 12)
        out = np.zeros_like(pose_in)
        tr = np.zeros((count, self.iterations, self.B, 10), np.float32) if trace else None
        rc = L.oracle_solve(self.h, first, count, _ptr(pose_in), _ptr(targets), _ptr(out), _ptr(tr), threads)
        if rc != 0:
            raise RuntimeError(f"oracle_solve failed rc={rc}")
        return (out, tr) if trace else out

    def segment_count(self):
        return lib().oracle_segment_count(self.h)

    def bone_list(self):
        buf = np.zeros(self.B, np.int32)
        n = lib().oracle_bone_list(self.h, _ptr(buf), self.B)
        return buf[:n].tolist()

    def segment_table(self):
        cap = self.B
        r = np.zeros(cap, np.int32); t = np.zeros(cap, np.int32); nh = np.zeros(cap, np.int32)
        n = lib().oracle_segment_table(self.h, _ptr(r), _ptr(t), _ptr(nh), cap)
        return r[:n], t[:n], nh[:n]

    def segment_solve(self, post_index, pose, targets, first=0):
        pose = np.ascontiguousarray(pose, np.float32).copy()
        targets = np.ascontiguousarray(targets, np.float32)
        rc = lib().oracle_segment_solve(self.h, post_index, first, pose.shape[0], _ptr(pose), _ptr(targets))
        if rc != 0:
            raise RuntimeError("oracle_segment_solve failed")
        return pose

    def close(self):
        if self.h:
            lib().oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def qcp(moved, target, weight, translate, precision):
    m = np.ascontiguousarray(moved, np.float32).reshape(-1)
    t = np.ascontiguousarray(target, np.float32).reshape(-1)
    w = np.ascontiguousarray(weight, np.float64)
    q = np.zeros(4, np.float32)
    tr = np.zeros(3, np.float32)
    lib().oracle_qcp(m, t, w, w.shape[0], int(translate), float(precision), q, tr)
    return q, tr


def local_point_in_limits(cones, point, tangents=None):
    c = np.ascontiguousarray(cones, np.float32).reshape(-1)
    tg = None if tangents is None else np.ascontiguousarray(tangents, np.float32).reshape(-1)
    out = np.zeros(3, np.float32)
    ib = lib().oracle_local_point_in_limits(c, c.shape[0] // 4, _ptr(tg), np.ascontiguousarray(point, np.float32), out)
    return out, ib


def closest_path_point(cones, cone_index, use_next, point, tangents=None):
    c = np.ascontiguousarray(cones, np.float32).reshape(-1)
    tg = None if tangents is None else np.ascontiguousarray(tangents, np.float32).reshape(-1)
    out = np.zeros(3, np.float32)
    lib().oracle_closest_path_point(c, c.shape[0] // 4, _ptr(tg), cone_index, use_next,
                                    np.ascontiguousarray(point, np.float32), out)
    return out


def cone_tangents(cones):
    c = np.ascontiguousarray(cones, np.float32).reshape(-1)
    out = np.zeros((c.shape[0] // 4, 8), np.float32)
    lib().oracle_cone_tangents(c, c.shape[0] // 4, out)
    return out


def xform_mul(a, b):
    out = np.zeros(12, np.float32)
    lib().oracle_xform_mul(np.ascontiguousarray(a, np.float32), np.ascontiguousarray(b, np.float32), out)
    return out


def xform_affine_inverse(a):
    out = np.zeros(12, np.float32)
    lib().oracle_xform_affine_inverse(np.ascontiguousarray(a, np.float32), out)
    return out


def libm_fill(fn: int, first: int, count: int, inputs: np.ndarray | None = None, threads: int = 8) -> np.ndarray:
    """Host platform-libm values of the device's transcendental call sites (libm_ref.c):
    float results for codes 0-3, double for 4-5 (codes as MBIK_LIBM_* in include/mbik.h)."""
    out = np.empty(count, np.float32 if fn <= 3 else np.float64)
    if inputs is not None:
        inputs = np.ascontiguousarray(inputs, np.float64)
    rc = lib().oracle_libm_fill(fn, first, count, _ptr(inputs), out.ctypes.data, threads)
    assert rc == 0
    return out


def libm_restated_mismatches(fn: int, first: int, count: int, stride: int = 1):
    """glibc_libm.h vs the platform libm (codes 0-2) on `count` inputs first, first+stride, ...:
    (mismatches, first mismatching bit pattern or None)."""
    fb = C.c_uint64(0)
    n = int(lib().oracle_libm_restated_mismatches(fn, first, count, stride, C.byref(fb)))
    return n, (int(fb.value) if n else None)
