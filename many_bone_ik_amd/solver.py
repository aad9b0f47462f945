"""Host-side plan/solve wrapper over the C ABI (include/mbik.h).

`Plan` owns one `mbik_plan` (topology tables + per-skeleton setup data resident on one
GPU).  `solve()` takes device pointers (e.g. torch CUDA tensors' data_ptr()) and is
asynchronous on the given HIP stream; `solve_host()` takes numpy arrays.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import MbikConfig, MbikConstraint, MbikPin, MbikPlanInfo, MbikPlanOptions, MbikSkeletonDesc, check


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class _Desc:
    """Keeps the ctypes structures (and the arrays they point into) alive together."""

    def __init__(self, parents, pins, constraints, max_cones, iterations, default_damp, constraint_mode,
                 stabilization_passes, bone_damp):
        self.parents = np.ascontiguousarray(parents, np.int32)
        B = self.parents.shape[0]
        self.pin_arr = (MbikPin * max(1, len(pins)))()
        for i, p in enumerate(pins):
            self.pin_arr[i].bone = int(p["bone"])
            self.pin_arr[i].weight = float(p.get("weight", 0.0))
            pr = p.get("direction_priorities", (0.2, 0.0, 0.2))
            for a in range(3):
                self.pin_arr[i].direction_priorities[a] = float(pr[a])
            self.pin_arr[i].motion_propagation_factor = float(p.get("motion_propagation_factor", 1.0))
        self.con_arr = (MbikConstraint * max(1, len(constraints)))()
        for i, c in enumerate(constraints):
            self.con_arr[i].bone = int(c["bone"])
            self.con_arr[i].cone_count = int(c.get("cone_count", 0))
        d = MbikSkeletonDesc()
        d.bone_count = B
        d.parents = self.parents.ctypes.data_as(C.POINTER(C.c_int32))
        d.pin_count = len(pins)
        d.pins = C.cast(self.pin_arr, C.POINTER(MbikPin))
        d.constraint_count = len(constraints)
        d.constraints = C.cast(self.con_arr, C.POINTER(MbikConstraint))
        d.max_cones = int(max_cones)
        self.desc = d
        cfg = MbikConfig()
        cfg.iterations_per_frame = int(iterations)
        cfg.default_damp = float(default_damp)
        cfg.constraint_mode = int(bool(constraint_mode))
        cfg.stabilization_passes = int(stabilization_passes)
        self.bd = None if bone_damp is None else np.ascontiguousarray(bone_damp, np.float32)
        cfg.bone_damp_count = 0 if self.bd is None else self.bd.shape[0]
        cfg.bone_damp = None if self.bd is None else self.bd.ctypes.data_as(C.POINTER(C.c_float))
        self.cfg = cfg


def describe_topology(parents, pins, constraints=(), *, iterations=15, default_damp=math.radians(5.0),
                      bone_damp=None) -> dict:
    """Host-only segmentation (mbik_describe_topology): bone_list + post-order segment table."""
    L = _lib.load()
    constraints = list(constraints)
    mc = max([1] + [int(c.get("cone_count", 0)) for c in constraints])
    d = _Desc(parents, pins, constraints, mc, iterations, default_damp, False, 0, bone_damp)
    B = d.parents.shape[0]
    bl = np.zeros(B, np.int32); nbl = C.c_int32(0)
    r = np.zeros(B, np.int32); t = np.zeros(B, np.int32); p = np.zeros(B, np.int32); nh = np.zeros(B, np.int32)
    ns = check(L.mbik_describe_topology(C.byref(d.desc), C.byref(d.cfg), _ptr(bl), C.byref(nbl), _ptr(r), _ptr(t),
                                        _ptr(p), _ptr(nh)))
    return dict(bone_list=bl[:nbl.value], seg_root=r[:ns], seg_tip=t[:ns], seg_parent=p[:ns], seg_headings=nh[:ns])


def _rig_arrays(rigs):
    """ctypes arrays of descs / configs for (parents, pins, constraints, config-kwargs) rigs;
    returns (descs, configs, keepalive)."""
    keep = []
    descs = (MbikSkeletonDesc * len(rigs))()
    cfgs = (MbikConfig * len(rigs))()
    for i, (parents, pins, constraints, kw) in enumerate(rigs):
        constraints = list(constraints)
        mc = kw.get("max_cones", max([1] + [int(c.get("cone_count", 0)) for c in constraints]))
        d = _Desc(parents, pins, constraints, mc, kw.get("iterations", 15), kw.get("default_damp", math.radians(5.0)),
                  kw.get("constraint_mode", False), kw.get("stabilization_passes", 0), kw.get("bone_damp"))
        keep.append(d)
        descs[i] = d.desc
        cfgs[i] = d.cfg
    return descs, cfgs, keep


def topology_selftest(rigs, device: int = -1):
    """mbik_selftest_topology: builds the rigs' topologies with the GPU builder's code (on the
    host when device < 0) and compares every table with the host builder's.  Returns
    (per-rig mismatching table counts, the first difference's description)."""
    L = _lib.load()
    descs, cfgs, keep = _rig_arrays(rigs)
    out = (C.c_int32 * max(1, len(rigs)))()
    check(L.mbik_selftest_topology(len(rigs), descs, cfgs, int(device), out))
    return [int(out[i]) for i in range(len(rigs))], _lib.last_error()


def plans_from_device(rigs, n_skeletons, setup_pose_ptrs, cones_ptrs=None, twist_ptrs=None, device: int = 0,
                      libm_variant: int = 0):
    """mbik_plan_create_device: one Plan per rig, topology and setup built on the GPU from
    device buffers (setup poses, cones, twist: device pointers, 0 / None where a rig has no
    constraints)."""
    L = _lib.load()
    n = len(rigs)
    descs, cfgs, keep = _rig_arrays(rigs)
    vpa = C.c_void_p * n
    out = vpa()
    ptrs = lambda xs: vpa(*[(x or None) for x in (xs or [0] * n)])
    opts = MbikPlanOptions(C.sizeof(MbikPlanOptions), int(libm_variant))
    check(L.mbik_plan_create_device_opts(n, descs, cfgs, C.byref(opts), (C.c_int32 * n)(*n_skeletons), ptrs(setup_pose_ptrs),
                                         ptrs(cones_ptrs), ptrs(twist_ptrs), int(device), out))
    plans = []
    for i, (parents, pins, constraints, kw) in enumerate(rigs):
        p = Plan.__new__(Plan)
        p._L = L
        p.h = C.c_void_p(out[i])
        inf = p.info()
        p.n, p.B, p.P = inf["skeleton_count"], inf["bone_count"], inf["pin_count"]
        p._slots, p._cf_stride, p._cd_stride = inf["constraint_slots"], inf["cf_stride"], inf["cd_stride"]
        p.iterations = kw.get("iterations", 15)
        plans.append(p)
    return plans


class Plan:
    """== ManyBoneIK3D after _bone_list_changed(), for a batch of same-topology skeletons."""

    def __init__(self, parents, pins, constraints, setup_pose, cones=None, twist=None, *,
                 iterations=15, default_damp=math.radians(5.0), constraint_mode=False,
                 stabilization_passes=0, bone_damp=None, max_cones=None, device=0, lanes=0, libm_variant=0):
        L = _lib.load()
        self._L = L
        setup_pose = np.ascontiguousarray(setup_pose, np.float32)
        n, B = setup_pose.shape[0], np.asarray(parents).shape[0]
        assert setup_pose.shape == (n, B, 10), setup_pose.shape
        mc = max_cones if max_cones is not None else (cones.shape[2] if cones is not None and np.ndim(cones) == 4 else 1)
        d = _Desc(parents, pins, list(constraints), mc, iterations, default_damp, constraint_mode,
                  stabilization_passes, bone_damp)
        cones_a = None if cones is None else np.ascontiguousarray(cones, np.float32)
        twist_a = None if twist is None else np.ascontiguousarray(twist, np.float32)
        h = C.c_void_p()
        opts = MbikPlanOptions(C.sizeof(MbikPlanOptions), int(libm_variant))
        check(L.mbik_plan_create_opts(C.byref(d.desc), C.byref(d.cfg), C.byref(opts), n, _ptr(setup_pose), _ptr(cones_a),
                                      _ptr(twist_a), int(device), C.byref(h)))
        self.h = h
        self.n = n
        self.B = B
        # constraint slots = constraints whose bone is in the IK bone list (plan.cpp)
        bl = set(describe_topology(parents, pins, constraints, iterations=iterations, default_damp=default_damp,
                                   bone_damp=bone_damp)["bone_list"].tolist())
        self._slots = len({int(c["bone"]) for c in constraints if int(c["bone"]) in bl})
        self._cf_stride = 14 + 31 * max(1, int(mc))
        self._cd_stride = 2 * max(1, int(mc))
        self.P = len(pins)
        self.iterations = int(iterations)
        if lanes:
            self.set_launch(lanes)

    @classmethod
    def from_workload(cls, wl, device=0, lanes=0, iterations=None, stabilization_passes=0, constraint_mode=False,
                      libm_variant=0):
        t = wl.topo
        return cls(t.parents, wl.pins(), wl.constraints(), wl.pose, wl.cones, wl.twist,
                   iterations=t.iterations if iterations is None else iterations,
                   default_damp=wl.default_damp, max_cones=wl.cones.shape[2], device=device, lanes=lanes,
                   bone_damp=wl.bone_damp, stabilization_passes=stabilization_passes,
                   constraint_mode=constraint_mode, libm_variant=libm_variant)

    def save(self) -> bytes:
        """mbik_plan_save: the plan as a flat binary (topology inputs, setup tables, layout,
        constraint_mode node caches)."""
        size = C.c_uint64(0)
        check(self._L.mbik_plan_save(self.h, None, 0, C.byref(size)))
        buf = C.create_string_buffer(size.value)
        check(self._L.mbik_plan_save(self.h, buf, size.value, C.byref(size)))
        return buf.raw[: size.value]

    @classmethod
    def load(cls, data: bytes, device: int = 0) -> "Plan":
        """mbik_plan_load: a plan rebuilt on `device` from Plan.save() bytes."""
        L = _lib.load()
        h = C.c_void_p()
        check(L.mbik_plan_load(data, len(data), int(device), C.byref(h)))
        self = cls.__new__(cls)
        self._L = L
        self.h = h
        inf = self.info()
        self.n, self.B, self.P = inf["skeleton_count"], inf["bone_count"], inf["pin_count"]
        self._slots, self._cf_stride, self._cd_stride = inf["constraint_slots"], inf["cf_stride"], inf["cd_stride"]
        self.iterations = None
        return self

    def info(self) -> dict:
        inf = MbikPlanInfo()
        check(self._L.mbik_plan_get_info(self.h, C.byref(inf)))
        return {f: getattr(inf, f) for f, _ in MbikPlanInfo._fields_}

    def set_launch(self, lanes: int):
        check(self._L.mbik_plan_set_launch(self.h, int(lanes)))

    def set_layout(self, lanes: int = 0, skeletons_per_block: int = 0, global_checkpoint_interval: int = 0):
        """Launch layout override (0 = automatic); results do not depend on it."""
        check(self._L.mbik_plan_set_layout(self.h, int(lanes), int(skeletons_per_block),
                                           int(global_checkpoint_interval)))

    def set_heading_staging(self, staging: int = -1):
        """mbik_plan_set_heading_staging: 1 stage multi-effector segments' headings in LDS,
        0 every lane solves such a segment alone, 2 stage only the translating root segments,
        3 only segments with two or more effectors, 4 split-exchange (lanes build alternate
        effectors' headings and read each other's cross-lane; two-waves-per-SIMD build only),
        5 root segments as 2 and the rest as 4, -1 automatic; results do not depend on it."""
        check(self._L.mbik_plan_set_heading_staging(self.h, int(staging)))

    def set_locals_placement(self, placement: int = -1):
        """mbik_plan_set_locals_placement: 0 state in LDS, 1 bone locals in device memory,
        2 all per-skeleton state in device memory, -1 automatic."""
        check(self._L.mbik_plan_set_locals_placement(self.h, int(placement)))

    def set_waves_per_simd(self, waves: int = -1):
        """mbik_plan_set_waves_per_simd: 1 or 2 waves per SIMD, -1 automatic."""
        check(self._L.mbik_plan_set_waves_per_simd(self.h, int(waves)))

    def set_helper_wave(self, helper: int = -1):
        """mbik_plan_set_helper_wave: 1 a second wave per block computes each bone-step's
        parent-side work one step ahead (fully resident placement-0 launches), 0 off,
        -1 automatic."""
        check(self._L.mbik_plan_set_helper_wave(self.h, int(helper)))

    def set_wave_roles(self, roles: int = -1):
        """mbik_plan_set_wave_roles: 1 one wave per segment role and a lane per skeleton
        (64 skeletons per block, whole state in device memory), 0 off, -1 automatic."""
        check(self._L.mbik_plan_set_wave_roles(self.h, int(roles)))

    def status(self) -> int:
        """mbik_plan_status: MBIK_STATUS_HELPER_TIMEOUT (1) when a completed helper-wave launch of
        this plan timed out in the two-wave handshake, else 0 (not cleared by reading)."""
        st = C.c_uint32(0)
        check(self._L.mbik_plan_status(self.h, C.byref(st)))
        return int(st.value)

    def debug_helper(self, drop_record: int = -1, timeout_us: int = 0):
        """mbik_plan_debug_helper (test hook): the helper wave stops before record drop_record
        (-1 never); the handshake deadline in microseconds (0 = the default two seconds)."""
        check(self._L.mbik_plan_debug_helper(self.h, int(drop_record), int(timeout_us)))

    def set_table_addressing(self, wide: int = 0):
        """mbik_plan_set_table_addressing: 0 automatic (32-bit offsets below 4 GiB), 1 64-bit indices."""
        check(self._L.mbik_plan_set_table_addressing(self.h, int(wide)))

    def autotune(self, pose_in_ptr: int, targets_ptr: int, pose_out_ptr: int, first: int = 0,
                 count: int | None = None, stream: int = 0):
        """mbik_plan_autotune: time candidate layouts on this batch, keep the fastest."""
        count = self.n - first if count is None else count
        check(self._L.mbik_plan_autotune(self.h, first, count, C.c_void_p(pose_in_ptr), C.c_void_p(targets_ptr),
                                         C.c_void_p(pose_out_ptr), C.c_void_p(stream or None)))

    def rebuild_setup(self, setup_pose_ptr: int, cones_ptr: int = 0, twist_ptr: int = 0, first: int = 0,
                      count: int | None = None, stream: int = 0):
        """mbik_plan_rebuild_setup: re-derive the per-skeleton setup data on the GPU."""
        count = self.n - first if count is None else count
        check(self._L.mbik_plan_rebuild_setup(self.h, first, count, C.c_void_p(setup_pose_ptr),
                                              C.c_void_p(cones_ptr or None), C.c_void_p(twist_ptr or None),
                                              C.c_void_p(stream or None)))

    def setup_tables(self):
        """(D, CF, CD) per-skeleton setup tables as numpy arrays (mbik_plan_setup_tables)."""
        inf = self.info()
        n, B = inf["skeleton_count"], inf["bone_count"]
        D = np.zeros((B, 9, n), np.float32)
        slots, cfs, cds = inf["constraint_slots"], inf["cf_stride"], inf["cd_stride"]
        assert (slots, cfs, cds) == (self._slots, self._cf_stride, self._cd_stride)  # mbik.h's documented formula
        CF = np.zeros((slots, cfs, n), np.float32)
        CD = np.zeros((slots, cds, n), np.float64)
        check(self._L.mbik_plan_setup_tables(self.h, _ptr(D), _ptr(CF) if slots else None, _ptr(CD) if slots else None))
        return D, CF, CD

    def solve(self, pose_in_ptr: int, targets_ptr: int, pose_out_ptr: int, first: int = 0, count: int | None = None,
              stream: int = 0):
        count = self.n - first if count is None else count
        check(self._L.mbik_solve(self.h, first, count, C.c_void_p(pose_in_ptr), C.c_void_p(targets_ptr),
                                 C.c_void_p(pose_out_ptr), C.c_void_p(stream or None)))

    def solve_checked(self, pose_in_ptr: int, targets_ptr: int, pose_out_ptr: int, nonfinite_ptr: int, first: int = 0,
                      count: int | None = None, stream: int = 0):
        """mbik_solve_checked: also writes one byte per skeleton, 1 where a non-finite basis was
        output as the identity rotation (ik_bone_3d.cpp:174-176)."""
        count = self.n - first if count is None else count
        check(self._L.mbik_solve_checked(self.h, first, count, C.c_void_p(pose_in_ptr), C.c_void_p(targets_ptr),
                                         C.c_void_p(pose_out_ptr), C.c_void_p(nonfinite_ptr), C.c_void_p(stream or None)))

    def capture_targets(self, skeleton_global_ptr: int, target_global_ptr: int, targets_ptr: int,
                        visible_ptr: int = 0, first: int = 0, count: int | None = None, stream: int = 0):
        """mbik_capture_targets: skeleton-space targets from scene-space transforms."""
        count = self.n - first if count is None else count
        check(self._L.mbik_capture_targets(self.h, first, count, C.c_void_p(skeleton_global_ptr),
                                           C.c_void_p(target_global_ptr), C.c_void_p(visible_ptr or None),
                                           C.c_void_p(targets_ptr), C.c_void_p(stream or None)))

    def segment_solve(self, segment: int, pose_ptr: int, targets_ptr: int, first: int = 0, count: int | None = None,
                      stream: int = 0):
        count = self.n - first if count is None else count
        check(self._L.mbik_segment_solve(self.h, segment, first, count, C.c_void_p(pose_ptr), C.c_void_p(targets_ptr),
                                         C.c_void_p(stream or None)))

    def solve_host(self, pose_in, targets, first: int = 0) -> np.ndarray:
        pose_in = np.ascontiguousarray(pose_in, np.float32)
        targets = np.ascontiguousarray(targets, np.float32)
        count = pose_in.shape[0]
        assert pose_in.shape == (count, self.B, 10)
        assert targets.shape == (count, self.P, 12)
        out = np.empty_like(pose_in)
        check(self._L.mbik_solve_host(self.h, first, count, _ptr(pose_in), _ptr(targets), _ptr(out)))
        return out

    def segment_table(self):
        n = self.info()["segment_count"]
        r = np.zeros(n, np.int32); t = np.zeros(n, np.int32); p = np.zeros(n, np.int32)
        check(self._L.mbik_plan_segment_table(self.h, _ptr(r), _ptr(t), _ptr(p), n))
        return r, t, p

    def close(self):
        if getattr(self, "h", None):
            self._L.mbik_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Group:
    """mbik_group_*: several plans (distinct rigs) solved by one launch per frame."""

    def __init__(self, plans):
        self._L = _lib.load()
        self.plans = list(plans)            # keeps the plans alive while the group exists
        arr = (C.c_void_p * len(self.plans))(*[p.h for p in self.plans])
        h = C.c_void_p()
        check(self._L.mbik_group_create(arr, len(self.plans), C.byref(h)))
        self.h = h

    def solve(self, pose_in_ptrs, targets_ptrs, pose_out_ptrs, first=None, count=None, stream: int = 0):
        """Device pointers per plan; first / count: per-plan lists or None (whole plans)."""
        n = len(self.plans)
        vpa = C.c_void_p * n
        i32 = C.c_int32 * n
        f = i32(*first) if first is not None else None
        c = i32(*count) if count is not None else None
        check(self._L.mbik_group_solve(self.h, f, c, vpa(*pose_in_ptrs), vpa(*targets_ptrs), vpa(*pose_out_ptrs),
                                       C.c_void_p(stream or None)))

    def close(self):
        if getattr(self, "h", None):
            self._L.mbik_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """mbik_multi_*: one batch sharded over several plans (one per GPU) in one process;
    contiguous shards in plan order, poses gathered to the root device (peer copies)."""

    def __init__(self, plans, root_device: int = 0, stage_all: bool = False):
        self._L = _lib.load()
        self.plans = list(plans)            # keeps the plans alive while the handle exists
        arr = (C.c_void_p * len(self.plans))(*[p.h for p in self.plans])
        h = C.c_void_p()
        check(self._L.mbik_multi_create(arr, len(self.plans), int(root_device),
                                        _lib.MBIK_MULTI_STAGE_ALL if stage_all else 0, C.byref(h)))
        self.h = h

    def skeletons(self):
        """(total skeletons, shard offsets)."""
        off = (C.c_int64 * (len(self.plans) + 1))()
        n = self._L.mbik_multi_skeletons(self.h, off)
        return int(n), [int(x) for x in off]

    def solve(self, pose_in_ptr: int, targets_ptr: int, pose_out_ptr: int, root_stream: int = 0):
        check(self._L.mbik_multi_solve(self.h, C.c_void_p(pose_in_ptr), C.c_void_p(targets_ptr),
                                       C.c_void_p(pose_out_ptr), C.c_void_p(root_stream or None)))

    def close(self):
        if getattr(self, "h", None):
            self._L.mbik_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def quat_error(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Per-bone sign-invariant quaternion error min(|q-r|_inf, |q+r|_inf)."""
    qa = a[..., 0:4].astype(np.float64)
    qb = b[..., 0:4].astype(np.float64)
    return np.minimum(np.abs(qa - qb).max(-1), np.abs(qa + qb).max(-1))
