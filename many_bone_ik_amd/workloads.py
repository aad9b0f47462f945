"""Seeded synthetic workloads for the batched solve.

The same arrays feed the HIP path, the oracle and the bench, so the generator is the
single source of inputs.  Everything is numpy; per-skeleton randomness comes from a
splitmix64 stream seeded with ``seed ^ (cfg << 40) ^ skeleton_index`` so any skeleton
can be regenerated on its own.

Draw order per skeleton (fixed; changing it changes every fixture):
  1. for every bone b:   L ~ U[0.8, 1.2], axis ~ S^2 (2 draws), angle ~ U[0, 15 deg]
  2. for every bone b:   perturbation axis ~ S^2 (2 draws), angle ~ U[0, 30 deg]
  3. constrained configs, for every parented bone b: helper vector ~ S^2 (2 draws)
  4. rest="realistic*" only, for every bone b: offset direction, roll, scale (7 draws,
     ``_realistic_rest``)

Pose layout  [skel][bone][10] = quaternion xyzw | position xyz | scale xyz  (float32)
Target layout [skel][pin][12] = basis rows r0 r1 r2 | origin            (float32)
Cones  [skel][constraint][cone][4] = centre xyz | radius ; twist [skel][constraint][2]
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

SEED = 20240807
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


class SplitMix64:
    """Vectorised splitmix64: one independent stream per array element."""

    def __init__(self, state: np.ndarray):
        self.state = np.asarray(state, dtype=np.uint64).copy()

    def next_u64(self) -> np.ndarray:
        with np.errstate(over="ignore"):
            self.state = self.state + _GOLDEN
            z = self.state
            z = (z ^ (z >> np.uint64(30))) * _M1
            z = (z ^ (z >> np.uint64(27))) * _M2
            return z ^ (z >> np.uint64(31))

    def uniform(self) -> np.ndarray:
        return (self.next_u64() >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)

    def unit_vector(self) -> np.ndarray:
        z = 2.0 * self.uniform() - 1.0
        phi = 2.0 * math.pi * self.uniform()
        r = np.sqrt(np.maximum(0.0, 1.0 - z * z))
        return np.stack([r * np.cos(phi), r * np.sin(phi), z], axis=-1)


@dataclasses.dataclass
class Topology:
    name: str
    parents: np.ndarray            # int32 [B]
    pins: np.ndarray               # int32 [P] pinned bones (leaf tips)
    constrained: np.ndarray        # int32 [C] bones carrying a Kusudama
    iterations: int
    twist: tuple[float, float] | None  # (min_angle, range) radians
    cones_per_bone: int


@dataclasses.dataclass
class Workload:
    topo: Topology
    n: int
    pose: np.ndarray      # float32 [n][B][10]
    targets: np.ndarray   # float32 [n][P][12]
    cones: np.ndarray     # float32 [n][C][max_cones][4]
    twist: np.ndarray     # float32 [n][C][2]
    default_damp: float = math.radians(5.0)
    pin_weight: np.ndarray | None = None        # [P] float32, default 1.0 (template default is 0)
    pin_priority: np.ndarray | None = None      # [P][3], default (0.2, 0, 0.2)
    pin_propagation: np.ndarray | None = None   # [P], default 1.0
    cone_count: np.ndarray | None = None        # [C] cones per constraint, default topo.cones_per_bone
    bone_damp: np.ndarray | None = None         # ManyBoneIK3D::bone_damp, default empty

    def __post_init__(self):
        P = int(self.topo.pins.shape[0])
        C = int(self.topo.constrained.shape[0])
        if self.pin_weight is None:
            self.pin_weight = np.ones(P, np.float32)
        if self.pin_priority is None:
            self.pin_priority = np.tile(np.array([0.2, 0.0, 0.2], np.float32), (P, 1))
        if self.pin_propagation is None:
            self.pin_propagation = np.ones(P, np.float32)
        if self.cone_count is None:
            self.cone_count = np.full(C, self.topo.cones_per_bone, np.int32)

    @property
    def bone_count(self) -> int:
        return int(self.topo.parents.shape[0])

    def pins(self) -> list[dict]:
        return [dict(bone=int(b), weight=float(self.pin_weight[i]),
                     direction_priorities=tuple(float(x) for x in self.pin_priority[i]),
                     motion_propagation_factor=float(self.pin_propagation[i]))
                for i, b in enumerate(self.topo.pins)]

    def constraints(self) -> list[dict]:
        return [dict(bone=int(b), cone_count=int(self.cone_count[i])) for i, b in enumerate(self.topo.constrained)]


def _chain(parents: list[int], start_parent: int, length: int) -> int:
    p = start_parent
    for _ in range(length):
        parents.append(p)
        p = len(parents) - 1
    return p


def _finger_lengths(cfg: int, count: int, lo: int, hi: int, total: int) -> list[int]:
    rng = SplitMix64(np.array([SEED ^ (cfg << 40) ^ 0xFFFFFFFF], dtype=np.uint64))
    lens = [lo + min(hi - lo, int(rng.uniform()[0] * (hi - lo + 1))) for _ in range(count)]
    while sum(lens) != total:
        i = min(count - 1, int(rng.uniform()[0] * count))
        if sum(lens) < total and lens[i] < hi:
            lens[i] += 1
        elif sum(lens) > total and lens[i] > lo:
            lens[i] -= 1
    return lens


def topology(cfg: int) -> Topology:
    """Topologies of BASELINE.json configs C1..C5 (bone / effector / segment counts of
    SURVEY.md §8).  C2-C5 hang their chains off a single branching root bone, so the
    root segment (which translates every bone it holds, ik_bone_segment_3d.cpp:217-222)
    is that one bone.  With SURVEY Appendix C's multi-bone spine as root segment the
    reference's own solve diverges geometrically (target headings are taken relative to
    the effector bone, ik_effector_3d.cpp:97): positions reach ~1e10 by iteration 16,
    where no float comparison means anything.  DESIGN.md records the measurement."""
    parents: list[int] = []
    tips: list[int] = []
    if cfg == 1:
        tips.append(_chain(parents, -1, 8))
        return Topology("c1_chain8", np.array(parents, np.int32), np.array(tips, np.int32),
                        np.zeros(0, np.int32), 8, None, 0)
    root = _chain(parents, -1, 1)
    if cfg in (2, 3):
        for length in (8, 8, 8, 7):
            tips.append(_chain(parents, root, length))
        B = len(parents)
        constrained = np.arange(1, B, dtype=np.int32) if cfg == 2 else np.zeros(0, np.int32)
        return Topology(f"c{cfg}_root_4chains_8887", np.array(parents, np.int32), np.array(tips, np.int32),
                        constrained, 16, (0.0, 2.0 * math.pi) if cfg == 2 else None, 2 if cfg == 2 else 0)
    if cfg == 4:
        for arm_len in (7, 8):
            arm = _chain(parents, root, arm_len)
            for _ in range(4):
                tips.append(_chain(parents, arm, 6))
        return Topology("c4_root_arms2_fingers8x6", np.array(parents, np.int32), np.array(tips, np.int32),
                        np.zeros(0, np.int32), 16, None, 0)
    if cfg == 5:
        lens = _finger_lengths(5, 16, 6, 14, 167)
        k = 0
        for _ in range(4):
            limb = _chain(parents, root, 8)
            for _ in range(4):
                tips.append(_chain(parents, limb, lens[k]))
                k += 1
        B = len(parents)
        return Topology("c5_root_limbs4x8_fingers16", np.array(parents, np.int32), np.array(tips, np.int32),
                        np.arange(1, B, dtype=np.int32), 16, (math.radians(-15.0), math.radians(60.0)), 2)
    raise ValueError(f"unknown config {cfg}")


def _quat_from_axis_angle(axis: np.ndarray, angle: np.ndarray) -> np.ndarray:
    s = np.sin(angle * 0.5)[..., None]
    return np.concatenate([axis * s, np.cos(angle * 0.5)[..., None]], axis=-1)


def _quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz], axis=-1)


def _quat_to_mat(q: np.ndarray) -> np.ndarray:
    x, y, z, w = np.moveaxis(q, -1, 0)
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
        np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)], -1),
        np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def _rotate(v: np.ndarray, axis: np.ndarray, angle: float) -> np.ndarray:
    c, s = math.cos(angle), math.sin(angle)
    return v * c + np.cross(axis, v) * s + axis * (np.sum(axis * v, -1, keepdims=True)) * (1 - c)


def custom_topology(parents, pins, constrained=(), cones_per_bone=0, twist=None, iterations=16,
                    name="custom") -> Topology:
    return Topology(name, np.asarray(parents, np.int32), np.asarray(pins, np.int32),
                    np.asarray(constrained, np.int32), int(iterations), twist, int(cones_per_bone))


REST_MODES = ("plus_y", "realistic", "realistic_unit_scale")


def _realistic_rest(rng: SplitMix64, n: int, B: int, length: np.ndarray, q_rest: np.ndarray):
    """Draw order step 4 (the realistic modes only, after steps 1-3 so the default
    stream is untouched), for every bone b:
      offset direction: tilt ~ U[0, 110 deg] away from +Y, azimuth ~ U[0, 2pi)  (2 draws)
      roll about the bone's own +Y ~ U[-180, 180 deg)                            (1 draw)
      uniform scale ~ U[0.8, 1.25], then per-axis factors ~ U[0.9, 1.1]          (4 draws)
    An imported humanoid's hips, clavicles and fingers sit off +Y, so
    update_default_bone_direction_transform (ik_bone_3d.cpp:57-93) takes the general arc
    branch; the rolls and non-uniform scales reach get_rotation_quaternion's
    orthonormalization and get_scale (ik_bone_3d.cpp:170-179)."""
    tilt = np.empty((n, B)); azim = np.empty((n, B)); roll = np.empty((n, B))
    scale = np.empty((n, B, 3))
    for b in range(B):
        tilt[:, b] = math.radians(110.0) * rng.uniform()
        azim[:, b] = 2.0 * math.pi * rng.uniform()
        roll[:, b] = math.radians(360.0) * rng.uniform() - math.pi
        s = 0.8 + 0.45 * rng.uniform()
        for k in range(3):
            scale[:, b, k] = s * (0.9 + 0.2 * rng.uniform())
    direction = np.stack([np.sin(tilt) * np.cos(azim), np.cos(tilt), np.sin(tilt) * np.sin(azim)], -1)
    pos = direction * length[..., None]
    y_axis = np.broadcast_to(np.array([0.0, 1.0, 0.0]), (n, B, 3))
    q = _quat_mul(q_rest, _quat_from_axis_angle(y_axis, roll))
    return pos, q, scale


def generate(cfg: int, n: int, first: int = 0, seed: int = SEED, topo: Topology | None = None,
             rest: str = "plus_y") -> Workload:
    """Generate skeletons [first, first+n) of config ``cfg`` (1..5), or of ``topo`` (then
    ``cfg`` only seeds the streams).  Constrained bones must not be parentless.

    ``rest="plus_y"`` (the default) puts every child at local (0, L, 0)
    with unit scale.  ``rest="realistic"`` takes child offsets in random directions, bone
    roll and non-uniform scale (``_realistic_rest``); the cones still centre on R_local*(+Y)
    and the targets are the FK (scale included) of the perturbed pose.
    ``rest="realistic_unit_scale"`` draws the same stream but keeps scale 1: on the long
    constrained C5 rig any non-unit scale makes the reference's own solve overflow within
    two iterations (the twist snap's P^-1 * orthonormalized(...) re-scales locals every step
    and the translating root segment amplifies it; DESIGN.md §7 records the probe), so C5's
    realistic fixture uses this mode."""
    if rest not in REST_MODES:
        raise ValueError(f"rest must be one of {REST_MODES}")
    topo = topology(cfg) if topo is None else topo
    B = topo.parents.shape[0]
    idx = np.arange(first, first + n, dtype=np.uint64)
    rng = SplitMix64(np.uint64(seed) ^ (np.uint64(cfg) << np.uint64(40)) ^ idx)
    length = np.empty((n, B)); rest_axis = np.empty((n, B, 3)); rest_angle = np.empty((n, B))
    for b in range(B):
        length[:, b] = 0.8 + 0.4 * rng.uniform()
        rest_axis[:, b] = rng.unit_vector()
        rest_angle[:, b] = math.radians(15.0) * rng.uniform()
    pert_axis = np.empty((n, B, 3)); pert_angle = np.empty((n, B))
    for b in range(B):
        pert_axis[:, b] = rng.unit_vector()
        pert_angle[:, b] = math.radians(30.0) * rng.uniform()
    q_rest = _quat_from_axis_angle(rest_axis, rest_angle)
    pos = np.zeros((n, B, 3))
    has_parent = topo.parents >= 0
    pos[:, has_parent, 1] = length[:, has_parent]
    scale = np.ones((n, B, 3))
    pose = np.zeros((n, B, 10), np.float32)

    C = topo.constrained.shape[0]
    helper = np.zeros((n, B, 3))
    if C:
        for b in range(B):
            if topo.parents[b] >= 0:
                helper[:, b] = rng.unit_vector()
    rest_dir = _quat_to_mat(q_rest)[..., :, 1]          # R_local * (0,1,0), parent frame (roll keeps it)
    if rest != "plus_y":
        r_pos, q_rest, r_scale = _realistic_rest(rng, n, B, length, q_rest)
        pos[:, has_parent] = r_pos[:, has_parent]
        if rest == "realistic":
            scale = r_scale
    pose[..., 0:4] = q_rest
    pose[..., 4:7] = pos
    pose[..., 7:10] = scale

    # Targets: FK of the perturbed pose; each pinned bone's global transform.
    q_pert = _quat_mul(_quat_from_axis_angle(pert_axis, pert_angle), q_rest)
    R = _quat_to_mat(q_pert) * scale[..., None, :]       # Basis(quat, scale): columns scaled
    G_R = np.empty((n, B, 3, 3)); G_o = np.empty((n, B, 3))
    order, seen = [], set()

    def visit(b):
        if b in seen:
            return
        if topo.parents[b] >= 0:
            visit(int(topo.parents[b]))
        seen.add(b)
        order.append(b)

    for b in range(B):
        visit(b)
    for b in order:
        p = topo.parents[b]
        if p < 0:
            G_R[:, b] = R[:, b]; G_o[:, b] = pos[:, b]
        else:
            G_R[:, b] = G_R[:, p] @ R[:, b]
            G_o[:, b] = G_o[:, p] + np.einsum("nij,nj->ni", G_R[:, p], pos[:, b])
    P = topo.pins.shape[0]
    targets = np.zeros((n, P, 12), np.float32)
    targets[..., 0:9] = G_R[:, topo.pins].reshape(n, P, 9)
    targets[..., 9:12] = G_o[:, topo.pins]

    C = topo.constrained.shape[0]
    mc = max(1, topo.cones_per_bone)
    cones = np.zeros((n, C, mc, 4), np.float32)
    twist = np.zeros((n, C, 2), np.float32)
    if C:
        cb = topo.constrained
        c0 = rest_dir[:, cb]
        perp = np.cross(c0, helper[:, cb])
        perp /= np.linalg.norm(perp, axis=-1, keepdims=True)
        c1 = _rotate(c0, perp, math.radians(45.0))
        cones[:, :, 0, 0:3] = c0
        cones[:, :, 0, 3] = math.radians(35.0)
        if topo.cones_per_bone > 1:
            cones[:, :, 1, 0:3] = c1
            cones[:, :, 1, 3] = math.radians(20.0)
        if topo.twist is not None:
            twist[..., 0] = topo.twist[0]
            twist[..., 1] = topo.twist[1]
    return Workload(topo, n, pose, targets, cones, twist)


def bench_config_name(cfg: int) -> str:
    return topology(cfg).name


# SURVEY.md §8's serial critical path per iteration on Appendix C's spine topologies
SURVEY_CRITICAL_PATH = {1: 8, 2: 11, 3: 11, 4: 16, 5: 30}


def critical_path_steps(topo: Topology) -> int:
    """Bone-steps per iteration on the longest root->leaf path of the IK bone list: the serial
    chain one iteration costs when sibling segments run concurrently (the post-order recursion
    of ik_bone_segment_3d.cpp:210-225 orders a segment after its children only).  Bones with no
    pinned descendant are not solved (ik_bone_segment_3d.cpp:390-393) and do not count."""
    B = topo.parents.shape[0]
    pinned = np.zeros(B, bool)
    for p in topo.pins:
        b = int(p)
        while b >= 0 and not pinned[b]:
            pinned[b] = True                 # bone b has a pinned descendant (or is pinned)
            b = int(topo.parents[b])
    best = 0
    for b in range(B):
        if not pinned[b]:
            continue
        d, a = 0, b
        while a >= 0:
            d += 1
            a = int(topo.parents[a])
        best = max(best, d)
    return best
