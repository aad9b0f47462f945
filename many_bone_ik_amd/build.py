"""Builds libmbik.so in-tree for gfx950 (hipcc, no JIT cache, no pip install).

    python -m many_bone_ik_amd.build [--force]

The library is rebuilt whenever the SHA-256 of its inputs -- every source, every header
under csrc/ and include/, and the compiler flags -- differs from the stamp written next to
it (libmbik.so.sha256), so an edited header can never leave a stale kernel in place.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmbik.so")
SOURCES = ["solve.hip", "plan.cpp"]
STAMP = OUT + ".sha256"

# -ffp-contract=off: every float op rounds separately, as the reference's x86 build does.
# -fno-slp-vectorize: the SLP vectorizer's packed fp32 ops cost more register copies than
# they save in this scalar chain (half the v_mov/v_accvgpr traffic without it; C3 -3%,
# C2 unchanged; tools/ab_run.sh).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-slp-vectorize",
         "-Wno-unused-result"]


def _inputs() -> list[str]:
    return sorted([os.path.join(CSRC, f) for f in SOURCES] + glob.glob(os.path.join(CSRC, "*.h")) +
                  glob.glob(os.path.join(HERE, "..", "include", "*.h")), key=os.path.basename)


def source_hash(extra_flags=()) -> str:
    h = hashlib.sha256(" ".join(FLAGS + list(extra_flags)).encode())
    for f in _inputs():
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale() -> bool:
    """True unless libmbik.so exists and was built from exactly the current inputs."""
    if not os.path.exists(OUT) or not os.path.exists(STAMP):
        return True
    with open(STAMP) as fh:
        return fh.read().strip() != source_hash()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, *[os.path.join(CSRC, f) for f in SOURCES], "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    digest = source_hash()
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    with open(STAMP, "w") as fh:
        fh.write(digest + "\n")
    return OUT


# tests/capi_frame.c: a C99 consumer of include/mbik.h (INTEGRATION.md §3's frame loop), linked
# against the in-tree libmbik.so through an $ORIGIN rpath so the binary travels with the tree.
CAPI_FRAME_SRC = os.path.join(HERE, "..", "tests", "capi_frame.c")
CAPI_FRAME = os.path.join(HERE, "..", "tests", "capi_frame")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def capi_frame_cmd(out: str = CAPI_FRAME) -> list[str]:
    return ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O2", "-D__HIP_PLATFORM_AMD__",
            "-I", os.path.join(HERE, "..", "include"), "-I", os.path.join(ROCM, "include"), CAPI_FRAME_SRC,
            "-L", HERE, "-l:libmbik.so", "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
            "-Wl,-rpath,$ORIGIN/../many_bone_ik_amd", "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-o", out]


def build_capi_frame(verbose: bool = False) -> str:
    build()
    src_newer = (not os.path.exists(CAPI_FRAME) or os.path.getmtime(CAPI_FRAME) < max(
        os.path.getmtime(CAPI_FRAME_SRC), os.path.getmtime(OUT), os.path.getmtime(os.path.join(HERE, "..", "include", "mbik.h"))))
    if src_newer:
        cmd = capi_frame_cmd()
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return CAPI_FRAME


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_capi_frame(verbose=True))
