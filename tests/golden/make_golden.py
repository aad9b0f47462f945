"""Regenerates the committed oracle fixtures in tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

Each fixture stores the generator coordinates (config, first skeleton, count), a SHA-256
of the generated inputs (so generator drift is caught), and the oracle's outputs:
full-frame poses, and for C1 (the reference's own CPU case) the pose after every
iteration.  The oracle is the plain-C restatement in oracle/; its transcendentals are the
platform libm's, glibc 2.35 (x86-64 FMA ifunc variant) -- what a Linux x86-64 Godot build
of the reference calls (oracle/godot_math.h; the 'libm' key records it).  SURVEY §7 hard part 1
and §8(c) ask every fixture to record the Godot-core version its arithmetic assumes (the
reference pins none; 'godot_version') and the oracle it came from ('oracle_sha256': SHA-256 of
the oracle's C sources, oracle_source_hash(); tests/test_oracle_golden.py checks it is current).
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from many_bone_ik_amd import workloads as W  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

LIBM = "glibc 2.35 platform libm (sinf/cosf/acosf FMA ifunc variant; tools/libm_exhaustive.c)"
# The reference ships no Godot version; SkeletonModifier3D / _process_modification imply >= 4.3, and
# the restated core math (Quaternion(v0, v1) normalizing its inputs) is 4.3's.
GODOT_VERSION = "4.3 (assumed: SkeletonModifier3D implies >= 4.3; Appendix B semantics restated from 4.3)"
ORACLE_SOURCES = ("ik_oracle.c", "godot_math.h", "glibc_libm.h", "mbik_oracle.h")


def oracle_source_hash() -> str:
    """SHA-256 over the oracle's C sources (name + bytes, in ORACLE_SOURCES order)."""
    h = hashlib.sha256()
    for f in ORACLE_SOURCES:
        h.update(f.encode())
        with open(os.path.join(ROOT, "oracle", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()
# (config, first skeleton, count, rest mode of workloads.generate)
FIXTURES = [(1, 0, 1, "plus_y"), (2, 0, 4, "plus_y"), (3, 0, 4, "plus_y"), (4, 0, 2, "plus_y"), (5, 0, 1, "plus_y"),
            (2, 4093, 3, "plus_y"),
            # off-+Y child offsets, bone roll, non-uniform scale: the bone-direction
            # arc's general branch (ik_bone_3d.cpp:57-93) and get_scale (:170-179)
            (2, 0, 4, "realistic"), (4, 0, 2, "realistic"), (5, 0, 1, "realistic_unit_scale")]


def fixture_name(cfg, first, n, rest):
    return f"oracle_c{cfg}_{first}_{n}.npz" if rest == "plus_y" else f"oracle_c{cfg}_{first}_{n}_{rest}.npz"


def generate(f):
    """The workload a loaded fixture was made from (fixtures before round 4 carry no 'rest')."""
    rest = str(f["rest"]) if "rest" in f else "plus_y"
    return W.generate(int(f["cfg"]), int(f["n"]), first=int(f["first"]), rest=rest)


def input_digest(wl) -> str:
    h = hashlib.sha256()
    for a in (wl.pose, wl.targets, wl.cones, wl.twist):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    for cfg, first, n, rest in FIXTURES:
        wl = W.generate(cfg, n, first=first, rest=rest)
        o = po.Oracle(wl)
        out, trace = o.solve(wl.pose, wl.targets, trace=True)
        seg_root, seg_tip, seg_nh = o.segment_table()
        # one segment_solver() call on the first (deepest) segment, from the input pose
        seg0 = o.segment_solve(0, wl.pose, wl.targets)
        name = os.path.join(HERE, fixture_name(cfg, first, n, rest))
        np.savez_compressed(name, cfg=cfg, first=first, n=n, rest=rest, digest=input_digest(wl), pose_out=out,
                            trace=trace if cfg == 1 else trace[:, :1], seg_root=seg_root, seg_tip=seg_tip,
                            seg_nh=seg_nh, libm=LIBM, bone_list=np.array(o.bone_list(), np.int32), segment0_pose=seg0,
                            godot_version=GODOT_VERSION, oracle_sha256=oracle_source_hash())
        print(name, os.path.getsize(name), "bytes")


if __name__ == "__main__":
    main()
