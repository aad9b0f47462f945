"""Host mirror of the reference's ManyBoneIK3D configuration surface (Python side).

The reference is a Godot SkeletonModifier3D (src/many_bone_ik_3d.{h,cpp}); its solve
path is replaced by the C ABI in include/mbik.h.  This class keeps the reference's
property names, defaults and index/ERR_FAIL behaviour (out-of-range indices are ignored,
getters return the reference's defaults) so code written against ManyBoneIK3D maps 1:1,
and it solves a whole batch of same-topology skeletons per `process_modification` call.

    ik = ManyBoneIK3D(parents, bone_names)
    ik.set_total_effector_count(2)
    ik.set_effector_bone_name(0, "hand_l"); ik.set_pin_weight(0, 1.0)
    ...
    pose_out = ik.process_modification(pose_in, targets)     # [n][bones][10] numpy
"""
from __future__ import annotations

import math

import numpy as np

from .solver import Plan, describe_topology


class ManyBoneIK3D:
    def __init__(self, parents, bone_names=None, device: int = 0):
        self.parents = np.asarray(parents, np.int32)
        B = self.parents.shape[0]
        self.bone_names = list(bone_names) if bone_names is not None else [f"bone_{i}" for i in range(B)]
        self.device = device
        # many_bone_ik_3d.h:49-68 defaults
        self.iterations_per_frame = 15
        self.default_damp = math.radians(5.0)
        self.constraint_mode = False
        self.stabilization_passes = 0
        self.bone_damp: list[float] = []
        # pins: IKEffectorTemplate3D defaults (ik_effector_template_3d.h:40-47)
        self._pins: list[dict] = []
        self._pin_count = 0          # pin_count: set_pin_count changes it without resizing pins (:58-60)
        self.ui_selected_bone = -1   # many_bone_ik_3d.h: editor selection, stored only
        self.node_exists = lambda path: True   # scene-tree lookup for set_effector_pin_node_path
        # constraints (many_bone_ik_3d.cpp:467-490 defaults for new entries)
        self._constraints: list[dict] = []
        self._plan: Plan | None = None
        self._dirty = True

    # ----------------------------------------------------------------- helpers
    def find_bone(self, name: str) -> int:
        try:
            return self.bone_names.index(name)
        except ValueError:
            return -1

    def set_dirty(self):
        self._dirty = True

    # ----------------------------------------------------------------- pins
    def set_total_effector_count(self, count: int):       # many_bone_ik_3d.cpp:44-52
        self._pin_count = int(count)
        while len(self._pins) < count:
            self._pins.append(dict(name="", weight=0.0, direction_priorities=(0.2, 0.0, 0.2),
                                   motion_propagation_factor=1.0, target_node=""))
        del self._pins[count:]
        self.set_dirty()

    def get_effector_count(self) -> int:                  # :54-56 (pin_count, not pins.size())
        return self._pin_count

    def set_effector_count(self, count: int):             # :58-60: the count only, no resize, not dirty
        self._pin_count = int(count)

    get_pin_count = get_effector_count                    # bound names (:400-401)
    set_pin_count = set_effector_count

    def find_pin(self, name: str) -> int:                 # :986-993, over pin_count
        for i in range(self._pin_count):
            if self.get_effector_bone_name(i) == name:
                return i
        return -1

    def get_pin_enabled(self, i: int) -> bool:            # :911-918: true for any valid index
        return 0 <= i < len(self._pins)

    def set_effector_pin_node_path(self, i: int, path: str):   # :629-637: only a path that resolves
        if 0 <= i < len(self._pins) and self.node_exists(path):
            self._pins[i]["target_node"] = str(path)

    def get_effector_pin_node_path(self, i: int) -> str:  # :639-643
        return self._pins[i]["target_node"] if 0 <= i < len(self._pins) else ""

    def set_effector_bone_name(self, i: int, bone: str):
        if 0 <= i < len(self._pins):
            self._pins[i]["name"] = bone
            self.set_dirty()

    def get_effector_bone_name(self, i: int) -> str:
        return self._pins[i]["name"] if 0 <= i < len(self._pins) else ""

    def set_pin_weight(self, i: int, weight: float):
        if 0 <= i < len(self._pins):
            self._pins[i]["weight"] = float(weight)
            self.set_dirty()

    def get_pin_weight(self, i: int) -> float:
        return self._pins[i]["weight"] if 0 <= i < len(self._pins) else 0.0

    def set_pin_direction_priorities(self, i: int, priorities):
        if 0 <= i < len(self._pins):
            self._pins[i]["direction_priorities"] = tuple(float(x) for x in priorities)
            self.set_dirty()

    def get_pin_direction_priorities(self, i: int):
        return self._pins[i]["direction_priorities"] if 0 <= i < len(self._pins) else (0.0, 0.0, 0.0)

    def set_pin_motion_propagation_factor(self, i: int, factor: float):
        if 0 <= i < len(self._pins):
            self._pins[i]["motion_propagation_factor"] = float(factor)
            self.set_dirty()

    def get_pin_motion_propagation_factor(self, i: int) -> float:
        return self._pins[i]["motion_propagation_factor"] if 0 <= i < len(self._pins) else 0.0

    def set_effector_target_node_path(self, i: int, path: str):   # many_bone_ik_3d.cpp:62-72
        if 0 <= i < len(self._pins):
            self._pins[i]["target_node"] = str(path)

    def get_effector_target_node_path(self, i: int) -> str:
        return self._pins[i]["target_node"] if 0 <= i < len(self._pins) else ""

    # ----------------------------------------------------------------- constraints
    def _set_constraint_count(self, count: int):           # many_bone_ik_3d.cpp:455-471
        while len(self._constraints) < count:
            self._constraints.append(dict(name="", cones=[(0.0, 1.0, 0.0, 0.01745)], cone_count=0,
                                          twist=(0.0, 0.01745)))
        del self._constraints[count:]
        self.set_dirty()

    def get_constraint_count(self) -> int:
        return len(self._constraints)

    set_constraint_count = _set_constraint_count          # bound name (:417)

    def find_constraint(self, name: str) -> int:          # :734-741
        for i, c in enumerate(self._constraints):
            if c["name"] == name:
                return i
        return -1

    def remove_constraint_at_index(self, i: int):         # :743-754
        if 0 <= i < len(self._constraints):
            del self._constraints[i]
            self.set_dirty()

    def set_constraint_name_at_index(self, i: int, name: str):
        if 0 <= i < len(self._constraints):
            self._constraints[i]["name"] = name
            self.set_dirty()

    def get_constraint_name(self, i: int) -> str:
        return self._constraints[i]["name"] if 0 <= i < len(self._constraints) else ""

    def set_kusudama_open_cone_count(self, i: int, count: int):   # :584-606
        if not 0 <= i < len(self._constraints):
            return
        c = self._constraints[i]
        cones = c["cones"]
        while len(cones) < count:
            cones.append((0.0, -1.0, 0.0, 0.0))  # forward_axis of an identity direction transform, 0 deg
        del cones[count:]
        c["cone_count"] = count
        self.set_dirty()

    def get_kusudama_open_cone_count(self, i: int) -> int:
        return self._constraints[i]["cone_count"] if 0 <= i < len(self._constraints) else 0

    def set_kusudama_open_cone_center(self, i: int, j: int, center):   # :578-592 (stored as given)
        if not 0 <= i < len(self._constraints):
            return
        cones = self._constraints[i]["cones"]
        if not 0 <= j < len(cones):
            return
        c = [float(x) for x in np.asarray(center, np.float32)]
        if abs(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) < 1e-5:   # Math::is_zero_approx(length_squared)
            c = [0.0, 1.0, 0.0]
        cones[j] = (c[0], c[1], c[2], cones[j][3])
        self.set_dirty()

    def set_kusudama_open_cone_radius(self, i: int, j: int, radius: float):   # :568-576
        if not 0 <= i < len(self._constraints):
            return
        c = self._constraints[i]
        if not (0 <= j < c["cone_count"] and j < len(c["cones"])):
            return
        cx, cy, cz, _ = c["cones"][j]
        c["cones"][j] = (cx, cy, cz, float(radius))
        self.set_dirty()

    def set_kusudama_open_cone(self, i: int, j: int, center, radius: float):
        """Convenience: set_kusudama_open_cone_center + set_kusudama_open_cone_radius."""
        self.set_kusudama_open_cone_center(i, j, center)
        self.set_kusudama_open_cone_radius(i, j, radius)

    def get_kusudama_open_cone_center(self, i: int, j: int):
        try:
            return self._constraints[i]["cones"][j][:3]
        except IndexError:
            return (0.0, 0.0, 1.0)

    def get_kusudama_open_cone_radius(self, i: int, j: int) -> float:
        try:
            return self._constraints[i]["cones"][j][3]
        except IndexError:
            return math.tau

    def set_joint_twist(self, i: int, twist):                      # :488-492
        if 0 <= i < len(self._constraints):
            self._constraints[i]["twist"] = (float(twist[0]), float(twist[1]))
            self.set_dirty()

    def get_joint_twist(self, i: int):
        return self._constraints[i]["twist"] if 0 <= i < len(self._constraints) else (0.0, 0.0)

    # ----------------------------------------------------------------- bone damp / reset
    def _set_bone_count(self, count: int):                # :756-764: new entries take default_damp
        while len(self.bone_damp) < count:
            self.bone_damp.append(self.default_damp)
        del self.bone_damp[count:]
        self.set_dirty()

    def get_bone_count(self) -> int:                      # :766-768
        return len(self.bone_damp)

    def reset_constraints(self):                          # :927-940 (the skeleton is always present)
        pins, cons = self._pin_count, len(self._constraints)
        self.set_total_effector_count(0)
        self.set_total_effector_count(pins)
        self._set_constraint_count(0)
        self._set_constraint_count(cons)
        self._set_bone_count(0)
        self._set_bone_count(cons)
        self.set_dirty()

    def register_skeleton(self):                          # :920-925
        if not self.get_effector_count() and not self.get_constraint_count():
            self.reset_constraints()
        self.set_dirty()

    def set_ui_selected_bone(self, bone: int):            # :950-956 (editor state, stored only)
        self.ui_selected_bone = int(bone)

    def get_ui_selected_bone(self) -> int:
        return self.ui_selected_bone

    # The per-bone IKNode3D transforms of the built tree (:774-909) are editor-gizmo accessors
    # of the reference's live object graph.  Here the tree lives on the device as the plan's
    # setup tables (mbik_plan_setup_tables); editing a node transform in place is not part of
    # the solve path this package replaces.
    def _tree_accessor(self, *_):
        raise NotImplementedError("IKNode3D transform accessors of the built tree are editor-gizmo helpers; "
                                  "read the plan's setup tables with Plan.setup_tables() (DESIGN.md §9)")

    get_twist_transform_of_constraint = set_twist_transform_of_constraint = _tree_accessor
    get_orientation_transform_of_constraint = set_orientation_transform_of_constraint = _tree_accessor
    get_direction_transform_of_bone = set_direction_transform_of_bone = _tree_accessor

    # ----------------------------------------------------------------- solver properties
    def set_iterations_per_frame(self, n):
        self.iterations_per_frame = int(n)
        self.set_dirty()

    def get_iterations_per_frame(self):
        return self.iterations_per_frame

    def set_default_damp(self, d):
        self.default_damp = float(d)
        self.set_dirty()

    def get_default_damp(self):
        return self.default_damp

    def set_constraint_mode(self, on: bool):
        self.constraint_mode = bool(on)
        self.set_dirty()

    def get_constraint_mode(self):
        return self.constraint_mode

    def set_stabilization_passes(self, n: int):
        self.stabilization_passes = int(n)
        self.set_dirty()

    def get_stabilization_passes(self):
        return self.stabilization_passes

    # ----------------------------------------------------------------- plan / solve
    def _pin_list(self):
        """Pins whose bone name resolves, in pin order (an unnamed or unknown-bone pin gets no
        effector, as the reference's segmentation finds no bone for it)."""
        return [dict(bone=self.find_bone(self._pins[i]["name"]), weight=self._pins[i]["weight"],
                     direction_priorities=self._pins[i]["direction_priorities"],
                     motion_propagation_factor=self._pins[i]["motion_propagation_factor"])
                for i in self._resolved_pin_indices()]

    def _resolved_pin_indices(self) -> list[int]:
        """Pin indices (into get_pin_count()'s list) that the plan's effectors stand for, in order."""
        return [i for i, p in enumerate(self._pins) if self.find_bone(p["name"]) >= 0]

    def _constraint_arrays(self, n: int):
        cons, cones, twist = [], [], []
        mc = max([1] + [c["cone_count"] for c in self._constraints])
        for c in self._constraints:
            b = self.find_bone(c["name"])
            if b < 0:
                continue
            cons.append(dict(bone=b, cone_count=c["cone_count"]))
            row = np.zeros((mc, 4), np.float32)
            for j in range(c["cone_count"]):
                row[j] = c["cones"][j]
            cones.append(row)
            twist.append(c["twist"])
        C = len(cons)
        cones_a = np.broadcast_to(np.array(cones, np.float32).reshape(1, C, mc, 4), (n, C, mc, 4)).copy() if C else None
        twist_a = np.broadcast_to(np.array(twist, np.float32).reshape(1, C, 2), (n, C, 2)).copy() if C else None
        return cons, cones_a, twist_a, mc

    def describe(self) -> dict:
        """Segmentation the next plan would use (no device needed)."""
        return describe_topology(self.parents, self._pin_list(), [], iterations=self.iterations_per_frame,
                                 default_damp=self.default_damp, bone_damp=self.bone_damp or None)

    def _bone_list_changed(self, setup_pose, cones=None, twist=None):
        """== ManyBoneIK3D::_bone_list_changed for a batch: (re)build the device plan."""
        n = setup_pose.shape[0]
        cons, cones_a, twist_a, mc = self._constraint_arrays(n)
        if cones is not None:
            cones_a = np.asarray(cones, np.float32)
        if twist is not None:
            twist_a = np.asarray(twist, np.float32)
        if self._plan is not None:
            self._plan.close()
        self._plan = Plan(self.parents, self._pin_list(), cons, setup_pose, cones_a, twist_a,
                          iterations=self.iterations_per_frame, default_damp=self.default_damp,
                          constraint_mode=self.constraint_mode, stabilization_passes=self.stabilization_passes,
                          bone_damp=self.bone_damp or None, max_cones=mc, device=self.device)
        self._dirty = False

    def process_modification(self, pose_in, targets, cones=None, twist=None):
        """== ManyBoneIK3D::_process_modification for every skeleton of the batch.

        pose_in [n][bones][10] and targets [n][pins][12] (numpy, host), one target row per pin
        index of get_pin_count()'s list, as each IKEffector3D reads its own target node.  Rows
        of pins whose bone does not resolve are ignored.  The plan is rebuilt from pose_in when
        dirty, exactly when the reference calls _bone_list_changed.
        """
        pose_in = np.ascontiguousarray(pose_in, np.float32)
        if self.get_effector_count() == 0 or not self._pins:   # :649-651 and the has_pins check (:669-678)
            return pose_in.copy()
        targets = np.asarray(targets, np.float32)
        if targets.ndim != 3 or targets.shape[0] != pose_in.shape[0] or targets.shape[1] != len(self._pins) \
                or targets.shape[2] != 12:
            raise ValueError(f"targets must be [n][{len(self._pins)} pins][12], got {targets.shape}")
        if self._dirty or self._plan is None or self._plan.n != pose_in.shape[0]:
            self._bone_list_changed(pose_in, cones, twist)
        resolved = self._resolved_pin_indices()
        if not resolved:                                        # no pin names a bone: nothing to solve
            return pose_in.copy()
        return self._plan.solve_host(pose_in, np.ascontiguousarray(targets[:, resolved]))
