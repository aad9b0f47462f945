"""Host mirror of ManyBoneIK3D's configuration API: defaults and index behaviour follow
src/many_bone_ik_3d.{h,cpp} and src/ik_effector_template_3d.h."""
import math

import numpy as np
import pytest

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


def test_every_bound_method_exists():
    """Every method ManyBoneIK3D binds to Godot (many_bone_ik_3d.cpp:378-427) has a mirror."""
    names = ["set_constraint_name_at_index", "set_total_effector_count", "get_twist_transform_of_constraint",
             "set_twist_transform_of_constraint", "get_orientation_transform_of_constraint",
             "set_orientation_transform_of_constraint", "get_direction_transform_of_bone",
             "set_direction_transform_of_bone", "remove_constraint_at_index", "register_skeleton", "reset_constraints",
             "set_dirty", "set_kusudama_open_cone_radius", "get_kusudama_open_cone_radius",
             "set_kusudama_open_cone_center", "get_kusudama_open_cone_center", "set_kusudama_open_cone_count",
             "get_kusudama_open_cone_count", "set_joint_twist", "get_joint_twist", "set_pin_motion_propagation_factor",
             "get_pin_motion_propagation_factor", "get_pin_count", "set_pin_count", "get_effector_bone_name",
             "get_pin_direction_priorities", "set_pin_direction_priorities", "get_effector_pin_node_path",
             "set_effector_pin_node_path", "set_pin_weight", "get_pin_weight", "get_pin_enabled", "get_constraint_name",
             "get_iterations_per_frame", "set_iterations_per_frame", "find_constraint", "find_pin",
             "get_constraint_count", "set_constraint_count", "get_default_damp", "set_default_damp", "get_bone_count",
             "set_constraint_mode", "get_constraint_mode", "set_ui_selected_bone", "get_ui_selected_bone",
             "set_stabilization_passes", "get_stabilization_passes", "set_effector_bone_name"]
    assert [n for n in names if not callable(getattr(ManyBoneIK3D, n, None))] == []


def test_pin_count_is_separate_from_the_pin_list():
    """set_pin_count (bound to set_effector_count, :58-60) changes pin_count only: the pin
    templates keep their size and find_pin scans pin_count entries (:986-993)."""
    ik = make()
    ik.set_total_effector_count(2)
    ik.set_effector_bone_name(0, "a3")
    ik.set_effector_bone_name(1, "b3")
    assert ik.get_pin_count() == 2 and ik.find_pin("b3") == 1 and ik.find_pin("hips") == -1
    ik.set_pin_count(1)
    assert ik.get_effector_count() == 1 and ik.find_pin("b3") == -1
    assert ik.get_effector_bone_name(1) == "b3"          # the template is still there
    assert ik.get_pin_enabled(1) and not ik.get_pin_enabled(2)


def test_constraint_find_remove_and_reset():
    ik = make()
    ik._set_constraint_count(3)
    for i, n in enumerate(["a1", "a2", "b1"]):
        ik.set_constraint_name_at_index(i, n)
    ik.set_kusudama_open_cone_count(1, 2)
    assert ik.find_constraint("a2") == 1 and ik.find_constraint("zz") == -1
    ik.remove_constraint_at_index(0)                      # :743-754 shifts the rest down
    assert ik.get_constraint_count() == 2 and ik.find_constraint("a2") == 0
    assert ik.get_kusudama_open_cone_count(0) == 2
    ik.remove_constraint_at_index(5)                      # ERR_FAIL_INDEX: ignored
    assert ik.get_constraint_count() == 2
    ik.set_total_effector_count(1)
    ik.set_effector_bone_name(0, "a3")
    ik.reset_constraints()                                # :927-940: counts kept, entries re-defaulted
    assert ik.get_constraint_count() == 2 and ik.get_constraint_name(0) == ""
    assert ik.get_effector_count() == 1 and ik.get_effector_bone_name(0) == ""
    assert ik.get_bone_count() == 2 and ik.bone_damp == [ik.get_default_damp()] * 2


def test_register_skeleton_and_editor_state():
    ik = make()
    ik.register_skeleton()                                # no pins, no constraints: reset, stays empty
    assert ik.get_effector_count() == 0 and ik.get_constraint_count() == 0
    ik.set_ui_selected_bone(3)
    assert ik.get_ui_selected_bone() == 3
    ik.set_total_effector_count(1)
    ik.node_exists = lambda path: path == "../Target"
    ik.set_effector_pin_node_path(0, "../Missing")        # get_node_or_null fails: ignored (:631-634)
    assert ik.get_effector_pin_node_path(0) == ""
    ik.set_effector_pin_node_path(0, "../Target")
    assert ik.get_effector_pin_node_path(0) == "../Target"


def test_process_modification_wants_one_target_row_per_pin():
    """targets are indexed by pin (get_pin_count()), resolved or not; a compacted array is an
    error before any device work."""
    ik = ManyBoneIK3D(np.array([-1, 0, 1], np.int32))
    ik.set_total_effector_count(2)
    ik.set_effector_bone_name(0, "bone_2")                 # pin 1 stays unnamed
    pose = np.zeros((3, 3, 10), np.float32)
    with pytest.raises(ValueError, match="2 pins"):
        ik.process_modification(pose, np.zeros((3, 1, 12), np.float32))
    assert ik._resolved_pin_indices() == [0]
