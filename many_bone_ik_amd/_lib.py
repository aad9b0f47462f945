"""ctypes bindings of the C ABI (include/mbik.h) exported by libmbik.so.

The product path always goes through this library: there is no CPU fallback.  If the
in-tree libmbik.so is missing the import of any solver entry point fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MBIK_LIB_OVERRIDE") or os.path.join(_HERE, "libmbik.so")  # override: ablation timing only

MBIK_OK = 0
MBIK_EINVAL = -1
MBIK_ENOMEM = -2
MBIK_EHIP = -3
MBIK_EUNSUPPORTED = -4
MBIK_ENODEV = -5
MBIK_MULTI_STAGE_ALL = 1

# mbik_selftest_libm function codes (include/mbik.h)
LIBM_SINF, LIBM_COSF, LIBM_ACOSF, LIBM_SLERP_SCALE0, LIBM_COS_F64_OF_F32, LIBM_COS_F64, LIBM_SINF_SSE2, LIBM_COSF_SSE2, \
    LIBM_SLERP_SCALE0_SSE2, LIBM_ACOSF_UNIT = range(10)
# mbik_plan_options.libm_variant: the reference host's glibc sinf/cosf build
LIBM_VARIANT_FMA, LIBM_VARIANT_SSE2 = 0, 1
# a process's environment that makes ITS glibc pick the SSE2 build (the reference host of LIBM_VARIANT_SSE2)
GLIBC_SSE2_TUNABLES = "glibc.cpu.hwcaps=-FMA,-AVX2_Usable"

EXPORTED_SYMBOLS = (
    "mbik_plan_create", "mbik_plan_create_opts", "mbik_plan_create_device_opts", "mbik_plan_destroy", "mbik_plan_save", "mbik_plan_load", "mbik_plan_get_info", "mbik_plan_set_launch", "mbik_plan_set_layout",
    "mbik_plan_autotune", "mbik_plan_resident_blocks", "mbik_plan_set_heading_staging",
    "mbik_plan_set_locals_placement", "mbik_plan_set_waves_per_simd", "mbik_plan_set_helper_wave", "mbik_plan_set_wave_roles", "mbik_plan_set_table_addressing", "mbik_plan_rebuild_setup", "mbik_plan_setup_tables",
    "mbik_plan_status", "mbik_plan_debug_helper",
    "mbik_solve", "mbik_solve_checked", "mbik_solve_host", "mbik_segment_solve", "mbik_plan_segment_table", "mbik_describe_topology",
    "mbik_group_create", "mbik_group_solve", "mbik_group_destroy", "mbik_multi_create", "mbik_multi_solve",
    "mbik_multi_skeletons", "mbik_multi_destroy", "mbik_capture_targets", "mbik_selftest_math",
    "mbik_selftest_libm", "mbik_selftest_div", "mbik_selftest_qcp", "mbik_selftest_point_in_limits", "mbik_selftest_xform", "mbik_selftest_topology", "mbik_plan_create_device", "mbik_last_error",
)


class MbikPin(C.Structure):
    _fields_ = [("bone", C.c_int32), ("weight", C.c_float), ("direction_priorities", C.c_float * 3),
                ("motion_propagation_factor", C.c_float)]


class MbikConstraint(C.Structure):
    _fields_ = [("bone", C.c_int32), ("cone_count", C.c_int32)]


class MbikSkeletonDesc(C.Structure):
    _fields_ = [("bone_count", C.c_int32), ("parents", C.POINTER(C.c_int32)),
                ("pin_count", C.c_int32), ("pins", C.POINTER(MbikPin)),
                ("constraint_count", C.c_int32), ("constraints", C.POINTER(MbikConstraint)),
                ("max_cones", C.c_int32)]


class MbikConfig(C.Structure):
    _fields_ = [("iterations_per_frame", C.c_int32), ("default_damp", C.c_float),
                ("constraint_mode", C.c_int32), ("stabilization_passes", C.c_int32),
                ("bone_damp_count", C.c_int32), ("bone_damp", C.POINTER(C.c_float))]


class MbikPlanInfo(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("skeleton_count", C.c_int32), ("bone_count", C.c_int32),
                ("pin_count", C.c_int32), ("segment_count", C.c_int32), ("level_count", C.c_int32),
                ("lanes_per_skeleton", C.c_int32), ("skeletons_per_block", C.c_int32),
                ("max_headings", C.c_int32), ("device", C.c_int32), ("device_bytes", C.c_int64),
                ("algorithmic_bytes_per_skeleton", C.c_double),
                ("algorithmic_flops_per_skeleton", C.c_double), ("lds_bytes_per_block", C.c_int64),
                ("checkpoint_interval", C.c_int32), ("heading_staging", C.c_int32), ("state_placement", C.c_int32),
                ("waves_per_simd", C.c_int32), ("constraint_slots", C.c_int32), ("cf_stride", C.c_int32),
                ("cd_stride", C.c_int32), ("libm_variant", C.c_int32),
                ("helper_wave", C.c_int32), ("heading_slots", C.c_int32), ("wave_roles", C.c_int32)]


class MbikPlanOptions(C.Structure):
    _fields_ = [("struct_size", C.c_int32), ("libm_variant", C.c_int32)]


class MbikError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mbik error {code}: {msg}")
        self.code = code


_lib = None


def load():
    """Load the in-tree libmbik.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        # torch's ROCm wheel bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).
        # Whichever is loaded first is shared by the process; torch only works on its own,
        # and libmbik's gfx950 code object runs on either, so let torch's load first.
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -m many_bone_ik_amd.build` "
                          "(the HIP path has no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.mbik_plan_create.argtypes = [C.POINTER(MbikSkeletonDesc), C.POINTER(MbikConfig), C.c_int32, vp, vp, vp, C.c_int32,
                                   C.POINTER(vp)]
    L.mbik_plan_create.restype = C.c_int32
    L.mbik_plan_create_opts.argtypes = [C.POINTER(MbikSkeletonDesc), C.POINTER(MbikConfig), C.POINTER(MbikPlanOptions), C.c_int32,
                                        vp, vp, vp, C.c_int32, C.POINTER(vp)]
    L.mbik_plan_create_opts.restype = C.c_int32
    L.mbik_plan_create_device_opts.argtypes = [C.c_int32, vp, vp, C.POINTER(MbikPlanOptions), C.POINTER(C.c_int32),
                                               C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.c_int32, C.POINTER(vp)]
    L.mbik_plan_create_device_opts.restype = C.c_int32
    L.mbik_plan_destroy.argtypes = [vp]
    L.mbik_plan_destroy.restype = None
    L.mbik_plan_save.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]
    L.mbik_plan_save.restype = C.c_int32
    L.mbik_plan_load.argtypes = [vp, C.c_uint64, C.c_int32, C.POINTER(vp)]
    L.mbik_plan_load.restype = C.c_int32
    L.mbik_plan_get_info.argtypes = [vp, C.POINTER(MbikPlanInfo)]
    L.mbik_plan_get_info.restype = C.c_int32
    L.mbik_plan_set_launch.argtypes = [vp, C.c_int32]
    L.mbik_plan_set_launch.restype = C.c_int32
    L.mbik_plan_set_layout.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.mbik_plan_set_layout.restype = C.c_int32
    L.mbik_plan_set_heading_staging.argtypes = [vp, C.c_int32]
    L.mbik_plan_set_heading_staging.restype = C.c_int32
    L.mbik_plan_set_locals_placement.argtypes = [vp, C.c_int32]
    L.mbik_plan_set_locals_placement.restype = C.c_int32
    L.mbik_plan_set_waves_per_simd.argtypes = [vp, C.c_int32]
    L.mbik_plan_set_waves_per_simd.restype = C.c_int32
    if hasattr(L, "mbik_plan_set_helper_wave"):  # (absent from older A/B builds)
        L.mbik_plan_set_helper_wave.argtypes = [vp, C.c_int32]
        L.mbik_plan_set_helper_wave.restype = C.c_int32
    if hasattr(L, "mbik_plan_set_wave_roles"):  # (ABI 8; absent from older A/B builds)
        L.mbik_plan_set_wave_roles.argtypes = [vp, C.c_int32]
        L.mbik_plan_set_wave_roles.restype = C.c_int32
    if hasattr(L, "mbik_plan_status"):  # (ABI 6; absent from older A/B builds)
        L.mbik_plan_status.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.mbik_plan_status.restype = C.c_int32
        L.mbik_plan_debug_helper.argtypes = [vp, C.c_int32, C.c_int32]
        L.mbik_plan_debug_helper.restype = C.c_int32
    if hasattr(L, "mbik_plan_set_table_addressing"):  # (absent from older A/B builds, tools/variant_check.py)
        L.mbik_plan_set_table_addressing.argtypes = [vp, C.c_int32]
        L.mbik_plan_set_table_addressing.restype = C.c_int32
    L.mbik_plan_autotune.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp]
    L.mbik_plan_autotune.restype = C.c_int32
    L.mbik_plan_resident_blocks.argtypes = [vp, C.c_int64]
    L.mbik_plan_resident_blocks.restype = C.c_int32
    L.mbik_plan_rebuild_setup.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp]
    L.mbik_plan_rebuild_setup.restype = C.c_int32
    L.mbik_plan_setup_tables.argtypes = [vp, vp, vp, vp]
    L.mbik_plan_setup_tables.restype = C.c_int32
    L.mbik_solve.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp]
    L.mbik_solve.restype = C.c_int32
    L.mbik_solve_checked.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp]
    L.mbik_solve_checked.restype = C.c_int32
    L.mbik_selftest_math.argtypes = [C.c_int32, C.POINTER(C.c_uint64)]
    L.mbik_selftest_math.restype = C.c_int32
    L.mbik_selftest_topology.argtypes = [C.c_int32, vp, vp, C.c_int32, C.POINTER(C.c_int32)]
    L.mbik_selftest_topology.restype = C.c_int32
    L.mbik_plan_create_device.argtypes = [C.c_int32, vp, vp, C.POINTER(C.c_int32), C.POINTER(vp), C.POINTER(vp),
                                          C.POINTER(vp), C.c_int32, C.POINTER(vp)]
    L.mbik_plan_create_device.restype = C.c_int32
    L.mbik_selftest_div.argtypes = [C.c_int32, C.c_uint64, C.POINTER(C.c_uint64)]
    L.mbik_selftest_div.restype = C.c_int32
    if hasattr(L, "mbik_selftest_qcp"):  # (ABI 8; absent from older A/B builds)
        fp = C.POINTER(C.c_float)
        L.mbik_selftest_qcp.argtypes = [C.c_int32, fp, fp, C.POINTER(C.c_double), C.c_int32, C.c_double, C.c_int32, fp]
        L.mbik_selftest_qcp.restype = C.c_int32
        L.mbik_selftest_point_in_limits.argtypes = [vp, C.c_int32, C.c_int32, fp, fp, C.POINTER(C.c_double)]
        L.mbik_selftest_point_in_limits.restype = C.c_int32
        L.mbik_selftest_xform.argtypes = [C.c_int32, fp, fp, C.c_int32, fp]
        L.mbik_selftest_xform.restype = C.c_int32
    L.mbik_selftest_libm.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, vp, vp, C.POINTER(C.c_uint64), vp]
    L.mbik_selftest_libm.restype = C.c_int32
    L.mbik_solve_host.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
    L.mbik_solve_host.restype = C.c_int32
    L.mbik_segment_solve.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp]
    L.mbik_segment_solve.restype = C.c_int32
    L.mbik_plan_segment_table.argtypes = [vp, vp, vp, vp, C.c_int32]
    L.mbik_plan_segment_table.restype = C.c_int32
    L.mbik_describe_topology.argtypes = [C.POINTER(MbikSkeletonDesc), C.POINTER(MbikConfig), vp, vp, vp, vp, vp, vp]
    L.mbik_describe_topology.restype = C.c_int32
    L.mbik_group_create.argtypes = [C.POINTER(vp), C.c_int32, C.POINTER(vp)]
    L.mbik_group_create.restype = C.c_int32
    L.mbik_group_solve.argtypes = [vp, vp, vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), vp]
    L.mbik_group_solve.restype = C.c_int32
    L.mbik_group_destroy.argtypes = [vp]
    L.mbik_group_destroy.restype = None
    if hasattr(L, "mbik_multi_create"):  # (ABI 8; absent from older A/B builds)
        L.mbik_multi_create.argtypes = [C.POINTER(vp), C.c_int32, C.c_int32, C.c_uint32, C.POINTER(vp)]
        L.mbik_multi_create.restype = C.c_int32
        L.mbik_multi_solve.argtypes = [vp, vp, vp, vp, vp]
        L.mbik_multi_solve.restype = C.c_int32
        L.mbik_multi_skeletons.argtypes = [vp, C.POINTER(C.c_int64)]
        L.mbik_multi_skeletons.restype = C.c_int64
        L.mbik_multi_destroy.argtypes = [vp]
        L.mbik_multi_destroy.restype = None
    L.mbik_capture_targets.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp]
    L.mbik_capture_targets.restype = C.c_int32
    L.mbik_last_error.argtypes = []
    L.mbik_last_error.restype = C.c_char_p
    _lib = L
    return L


def check(rc: int) -> int:
    if rc < 0:
        raise MbikError(rc, load().mbik_last_error().decode(errors="replace"))
    return rc


def last_error() -> str:
    """mbik_last_error() of this thread."""
    return load().mbik_last_error().decode(errors="replace")
