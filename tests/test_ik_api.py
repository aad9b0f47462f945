"""Host mirror of ManyBoneIK3D's configuration API: defaults and index behaviour follow
src/many_bone_ik_3d.{h,cpp} and src/ik_effector_template_3d.h."""
import math

import numpy as np

from many_bone_ik_amd.ik import ManyBoneIK3D


def make():
    parents = [-1, 0, 1, 2, 0, 4, 5]
    return ManyBoneIK3D(parents, ["hips", "a1", "a2", "a3", "b1", "b2", "b3"])


def test_defaults():
    ik = make()
    assert ik.get_iterations_per_frame() == 15
    assert abs(ik.get_default_damp() - math.radians(5.0)) < 1e-12
    assert ik.get_constraint_mode() is False and ik.get_stabilization_passes() == 0
    ik.set_total_effector_count(1)
    assert ik.get_pin_weight(0) == 0.0                       # template default weight 0
    assert ik.get_pin_direction_priorities(0) == (0.2, 0.0, 0.2)
    assert ik.get_pin_motion_propagation_factor(0) == 1.0
    ik._set_constraint_count(1)
    assert ik.get_joint_twist(0) == (0.0, 0.01745)
    assert ik.get_kusudama_open_cone_count(0) == 0


def test_out_of_range_is_ignored_like_err_fail_index():
    ik = make()
    ik.set_pin_weight(3, 1.0)
    assert ik.get_pin_weight(3) == 0.0
    assert ik.get_effector_bone_name(9) == ""
    assert ik.get_kusudama_open_cone_radius(0, 0) == math.tau


def test_cone_center_stored_as_given_and_zero_replaced():
    """set_kusudama_open_cone_center stores the vector as given (the cone setup normalizes
    it later, ik_open_cone_3d.cpp); a zero vector becomes +Y (many_bone_ik_3d.cpp:578-592)."""
    ik = make()
    ik._set_constraint_count(1)
    ik.set_kusudama_open_cone_count(0, 2)
    assert ik.get_kusudama_open_cone_center(0, 1) == (0.0, -1.0, 0.0)   # new cone: -Y of an identity frame
    assert ik.get_kusudama_open_cone_radius(0, 1) == 0.0
    ik.set_kusudama_open_cone(0, 0, (0, 0, 0), 0.3)
    ik.set_kusudama_open_cone(0, 1, (2, 0, 0), 0.2)
    assert ik.get_kusudama_open_cone_center(0, 0) == (0.0, 1.0, 0.0)
    assert ik.get_kusudama_open_cone_center(0, 1) == (2.0, 0.0, 0.0)
    ik.set_kusudama_open_cone_radius(0, 5, 1.0)  # out of range: ignored
    assert ik.get_kusudama_open_cone_radius(0, 1) == 0.2


def test_describe_segments(mbik):
    ik = make()
    ik.set_total_effector_count(2)
    ik.set_effector_bone_name(0, "a3")
    ik.set_effector_bone_name(1, "b3")
    d = ik.describe()
    assert d["seg_root"].tolist() == [1, 4, 0] and d["seg_tip"].tolist() == [3, 6, 0]
    assert d["bone_list"].tolist() == [3, 2, 1, 6, 5, 4, 0]
