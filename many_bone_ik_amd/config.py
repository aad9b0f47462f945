"""Config ingestion: ManyBoneIK3D properties as Godot stores them in a
scene, applied to the host mirror (many_bone_ik_amd.ik.ManyBoneIK3D) with the reference's
own `_set` / `_get` semantics (src/many_bone_ik_3d.cpp:118-375), quirks included:

* `_get` reports the twist as `constraints/<i>/twist_start` / `twist_end` (:262-267) but
  `_set` only accepts `twist_from` / `twist_range` (:334-341): a saved twist does not load
  back.  `apply_properties` reproduces that (the keys are ignored) unless
  `godot_twist_roundtrip=True` asks for the values to be honoured.
* A `pins/<i>/...` key with `i >= pin count` resizes the pins to the *constraint* count
  (:302-304), not to `i + 1`.
* `pins/<i>/target_static = true` clears the target node path (:312-316).
* `constraints/<i>/bone_direction`, `kusudama_orientation`, `kusudama_twist` (:359-370)
  act only on an already built segment tree; at scene load there is none, so they are
  ignored (the frames are derived from the setup pose by the plan build).

`parse_tscn` reads the `[node ... type="ManyBoneIK3D" ...]` sections of a text scene with
the Variant literals those properties use.
"""
from __future__ import annotations

import math
import re

from .ik import ManyBoneIK3D

__all__ = ["parse_variant", "parse_tscn", "apply_properties", "get_properties", "load_tscn"]


class StringName(str):
    """Godot StringName literal (&"...")."""


class NodePath(str):
    """Godot NodePath literal (NodePath("..."))."""


_CTOR = re.compile(r"^(Vector2|Vector3|Vector4|Quaternion|Transform3D|Basis|NodePath)\((.*)\)$", re.S)


def parse_variant(text: str):
    """Parses one Godot text-resource Variant literal (the subset ManyBoneIK3D uses)."""
    t = text.strip()
    if t in ("true", "false"):
        return t == "true"
    if t == "null":
        return None
    if t.startswith('&"') and t.endswith('"'):
        return StringName(_unescape(t[2:-1]))
    if t.startswith('"') and t.endswith('"'):
        return _unescape(t[1:-1])
    m = _CTOR.match(t)
    if m:
        kind, body = m.group(1), m.group(2).strip()
        if kind == "NodePath":
            return NodePath(_unescape(body.strip()[1:-1]) if body.startswith('"') else body)
        vals = tuple(float(x) for x in body.split(",")) if body else ()
        want = {"Vector2": 2, "Vector3": 3, "Vector4": 4, "Quaternion": 4, "Transform3D": 12, "Basis": 9}[kind]
        if len(vals) != want:
            raise ValueError(f"{kind} needs {want} components, got {len(vals)}: {text!r}")
        return vals
    try:
        return int(t)
    except ValueError:
        pass
    try:
        return float(t)
    except ValueError:
        pass
    if t in ("inf", "-inf", "nan"):
        return float(t)
    raise ValueError(f"unsupported Variant literal: {text!r}")


def _unescape(s: str) -> str:
    return s.replace('\\"', '"').replace("\\\\", "\\")


def parse_tscn(text: str, node_type: str = "ManyBoneIK3D") -> list[dict]:
    """Returns [{"name", "type", "parent", "properties": {key: value, ...}}] for every node of
    `node_type` in a .tscn text, properties in file order."""
    nodes = []
    cur = None
    pending_key, pending_val = None, ""
    for raw in text.splitlines():
        line = raw.rstrip()
        if pending_key is not None:  # multi-line value (balanced parentheses)
            pending_val += " " + line.strip()
            if pending_val.count("(") == pending_val.count(")"):
                cur["properties"][pending_key] = parse_variant(pending_val)
                pending_key = None
            continue
        if line.startswith("["):
            cur = None
            if line.startswith("[node "):
                attrs = dict(re.findall(r'(\w+)="((?:[^"\\]|\\.)*)"', line))
                if attrs.get("type") == node_type:
                    cur = {"name": attrs.get("name", ""), "type": node_type, "parent": attrs.get("parent", ""),
                           "properties": {}}
                    nodes.append(cur)
            continue
        if cur is None or not line.strip() or line.lstrip().startswith(";"):
            continue
        key, sep, val = line.partition("=")
        if not sep:
            continue
        key, val = key.strip(), val.strip()
        if key.startswith('"') and key.endswith('"'):
            key = key[1:-1]
        if val.count("(") != val.count(")"):
            pending_key, pending_val = key, val
            continue
        cur["properties"][key] = parse_variant(val)
    return nodes


def _slice(name: str, i: int) -> str:
    parts = name.split("/")
    return parts[i] if i < len(parts) else ""


def _to_int(s: str) -> int:
    m = re.match(r"^\s*-?\d+", s)  # String::to_int
    return int(m.group(0)) if m else 0


def apply_properties(ik: ManyBoneIK3D, props: dict, *, godot_twist_roundtrip: bool = False) -> list[str]:
    """== ManyBoneIK3D::_set for each (key, value) in order plus the bound properties
    (many_bone_ik_3d.cpp:429-433).  Returns the keys _set rejects (returns false for)."""
    ignored = []
    for name, value in props.items():
        if not _set(ik, str(name), value, godot_twist_roundtrip):
            ignored.append(str(name))
    return ignored


def _set(ik: ManyBoneIK3D, name: str, value, twist_roundtrip: bool) -> bool:
    bound = {"iterations_per_frame": lambda v: ik.set_iterations_per_frame(int(v)),
             "default_damp": lambda v: ik.set_default_damp(float(v)),
             "constraint_mode": lambda v: ik.set_constraint_mode(bool(v)),
             "stabilization_passes": lambda v: ik.set_stabilization_passes(int(v)),
             "ui_selected_bone": lambda v: None}
    if name in bound:
        bound[name](value)
        return True
    if name == "constraint_count":
        ik._set_constraint_count(int(value))
        return True
    if name == "pin_count":
        ik.set_total_effector_count(int(value))
        return True
    if name.startswith("pins/"):
        index, what = _to_int(_slice(name, 1)), _slice(name, 2)
        if index >= ik.get_effector_count():
            ik.set_total_effector_count(ik.get_constraint_count())  # as written (:302-304)
        if what == "bone_name":
            ik.set_effector_bone_name(index, str(value))
        elif what == "target_node":
            ik.set_effector_target_node_path(index, str(value))
        elif what == "target_static":
            if value:
                ik.set_effector_target_node_path(index, "")
        elif what == "motion_propagation_factor":
            ik.set_pin_motion_propagation_factor(index, float(value))
        elif what == "weight":
            ik.set_pin_weight(index, float(value))
        elif what == "direction_priorities":
            ik.set_pin_direction_priorities(index, tuple(float(x) for x in value))
        else:
            return False
        return True
    if name.startswith("constraints/"):
        index, what = _to_int(_slice(name, 1)), _slice(name, 2)
        begins = f"constraints/{index}/kusudama_open_cone/"
        if index >= ik.get_constraint_count():
            ik._set_constraint_count(ik.get_constraint_count())
        if what == "bone_name":
            ik.set_constraint_name_at_index(index, str(value))
        elif what == "twist_from":
            ik.set_joint_twist(index, (float(value), ik.get_joint_twist(index)[1]))
        elif what == "twist_range":
            ik.set_joint_twist(index, (ik.get_joint_twist(index)[0], float(value)))
        elif what in ("twist_start", "twist_end") and twist_roundtrip:
            tw = ik.get_joint_twist(index)
            ik.set_joint_twist(index, (float(value), tw[1]) if what == "twist_start" else (tw[0], float(value)))
        elif what == "kusudama_open_cone_count":
            ik.set_kusudama_open_cone_count(index, int(value))
        elif name.startswith(begins):
            cone_index, cone_what = _to_int(_slice(name, 3)), _slice(name, 4)
            if cone_what == "center":
                ik.set_kusudama_open_cone_center(index, cone_index, value)
            elif cone_what == "radius":
                ik.set_kusudama_open_cone_radius(index, cone_index, float(value))
            else:
                return False
        elif what in ("bone_direction", "kusudama_orientation", "kusudama_twist"):
            pass  # needs a built segment tree; none exists at load (module docstring)
        else:
            return False
        return True
    return False


def get_properties(ik: ManyBoneIK3D) -> dict:
    """== _get_property_list + _get (many_bone_ik_3d.cpp:118-292): the keys a scene save
    writes, twist reported as twist_start / twist_end."""
    out = {"iterations_per_frame": ik.get_iterations_per_frame(), "default_damp": ik.get_default_damp(),
           "constraint_mode": ik.get_constraint_mode(), "stabilization_passes": ik.get_stabilization_passes(),
           "pin_count": ik.get_effector_count()}
    for i in range(ik.get_effector_count()):
        out[f"pins/{i}/bone_name"] = StringName(ik.get_effector_bone_name(i))
        out[f"pins/{i}/target_node"] = NodePath(ik.get_effector_target_node_path(i))
        out[f"pins/{i}/target_static"] = ik.get_effector_target_node_path(i) == ""
        out[f"pins/{i}/motion_propagation_factor"] = ik.get_pin_motion_propagation_factor(i)
        out[f"pins/{i}/weight"] = ik.get_pin_weight(i)
        out[f"pins/{i}/direction_priorities"] = tuple(ik.get_pin_direction_priorities(i))
    out["constraint_count"] = ik.get_constraint_count()
    for i in range(ik.get_constraint_count()):
        out[f"constraints/{i}/bone_name"] = StringName(ik.get_constraint_name(i))
        tw = ik.get_joint_twist(i)
        out[f"constraints/{i}/twist_start"] = tw[0]
        out[f"constraints/{i}/twist_end"] = tw[1]
        out[f"constraints/{i}/kusudama_open_cone_count"] = ik.get_kusudama_open_cone_count(i)
        for j in range(ik.get_kusudama_open_cone_count(i)):
            out[f"constraints/{i}/kusudama_open_cone/{j}/center"] = tuple(ik.get_kusudama_open_cone_center(i, j))
            out[f"constraints/{i}/kusudama_open_cone/{j}/radius"] = ik.get_kusudama_open_cone_radius(i, j)
    return out


def format_variant(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, StringName):
        return '&"' + v.replace('"', '\\"') + '"'
    if isinstance(v, NodePath):
        return 'NodePath("' + v.replace('"', '\\"') + '")'
    if isinstance(v, str):
        return '"' + v.replace('"', '\\"') + '"'
    if isinstance(v, tuple):
        kind = {2: "Vector2", 3: "Vector3", 4: "Vector4", 12: "Transform3D"}[len(v)]
        return f"{kind}({', '.join(_num(x) for x in v)})"
    return _num(v)


def _num(x) -> str:
    if isinstance(x, int) and not isinstance(x, bool):
        return str(x)
    x = float(x)
    if math.isinf(x) or math.isnan(x):
        return str(x)
    r = repr(x)
    return r[:-2] if r.endswith(".0") else r


def load_tscn(text: str, parents, bone_names, node_name: str | None = None, device: int = 0,
              godot_twist_roundtrip: bool = False) -> ManyBoneIK3D:
    """Builds a ManyBoneIK3D mirror from the (first, or `node_name`) ManyBoneIK3D node of a
    .tscn text, for the skeleton given by `parents` / `bone_names`."""
    nodes = parse_tscn(text)
    if node_name is not None:
        nodes = [n for n in nodes if n["name"] == node_name]
    if not nodes:
        raise ValueError("no ManyBoneIK3D node in the scene")
    ik = ManyBoneIK3D(parents, bone_names, device=device)
    apply_properties(ik, nodes[0]["properties"], godot_twist_roundtrip=godot_twist_roundtrip)
    return ik
