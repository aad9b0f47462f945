"""Builds libmbik.so in-tree for gfx950 (hipcc, no JIT cache, no pip install).

    python -m many_bone_ik_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmbik.so")
SOURCES = ["solve.hip", "plan.cpp"]
HEADERS = ["gd_math.h", "plan.h", os.path.join("..", "..", "include", "mbik.h")]

# -ffp-contract=off: every float op rounds separately, as the reference's x86 build does.
# -fno-slp-vectorize: the SLP vectorizer's packed fp32 ops cost more register copies than
# they save in this scalar chain (half the v_mov/v_accvgpr traffic without it; C3 -3%,
# C2 unchanged; tools/ab_run.sh).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-slp-vectorize",
         "-Wno-unused-result"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, *[os.path.join(CSRC, f) for f in SOURCES], "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
