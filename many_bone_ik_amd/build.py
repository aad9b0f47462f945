"""Builds libmbik.so in-tree for gfx950 (hipcc, no JIT cache, no pip install).

    python -m many_bone_ik_amd.build [--force]
    python -m many_bone_ik_amd.build --variant OUT.so [-DNAME[=V] ...]   (diagnostic builds: tools/)

Every translation unit (the kernel families k_*.hip, the host side host_*.cpp and plan.cpp)
compiles to its own object in parallel, then one link.  The library is rebuilt whenever the
SHA-256 of its inputs -- every source, every header under csrc/ and include/, and the compiler
flags -- differs from the stamp written next to it (libmbik.so.sha256), so an edited header can
never leave a stale kernel in place.
"""
from __future__ import annotations

import concurrent.futures
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmbik.so")
# kernel families first (the longest compiles start first)
SOURCES = ["k_solve_w1.hip", "k_solve_w2.hip", "k_cmode.hip", "k_solve_rw.hip", "host_selftest.cpp", "k_aux.hip", "host_plan.cpp",
           "host_topo_io.cpp", "host_autotune.cpp", "host_multi.cpp", "plan.cpp"]
OBJ = os.path.join(HERE, "..", "build", "obj")
STAMP = OUT + ".sha256"

# -ffp-contract=off: every float op rounds separately, as the reference's x86 build does.
# -fno-slp-vectorize: the SLP vectorizer's packed fp32 ops cost more register copies than
# they save in this scalar chain (half the v_mov/v_accvgpr traffic without it; C3 -3%,
# C2 unchanged; tools/ab_run.sh).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-slp-vectorize",
         "-Wno-unused-result"]
COMPILE = [f for f in FLAGS if f != "-shared"]


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


def _jobs() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(int(os.environ.get("MAX_JOBS", "16")), n, len(SOURCES)))


def compile_library(out: str, extra_flags=(), verbose: bool = False, csrc: str = CSRC) -> None:
    """Compiles every translation unit of `csrc` (in parallel) and links them into `out`."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tag = hashlib.sha256((" ".join(COMPILE + list(extra_flags)) + out + csrc).encode()).hexdigest()[:12]
    odir = os.path.join(OBJ, tag)
    os.makedirs(odir, exist_ok=True)

    def one(src: str) -> str:
        obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *COMPILE, *extra_flags, "-c", os.path.join(csrc, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compiling {src} failed:\n{r.stderr}")
        return obj

    with concurrent.futures.ThreadPoolExecutor(_jobs()) as ex:
        objs = list(ex.map(one, SOURCES))
    cmd = [hipcc, *FLAGS, *extra_flags, *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    digest = source_hash()
    compile_library(OUT, verbose=verbose)
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
    if "--variant" in sys.argv:
        # a diagnostic build of the same sources with extra flags, e.g. -DMBIK_PROF (tools/)
        # (--csrc DIR: the sources of another revision, tools/ab_build.sh)
        args = sys.argv[sys.argv.index("--variant") + 1:]
        src = CSRC
        if "--csrc" in args:
            j = args.index("--csrc")
            src = os.path.abspath(args[j + 1])
            del args[j:j + 2]
        compile_library(os.path.abspath(args[0]), args[1:], verbose=True, csrc=src)
        print(args[0])
    else:
        print(build(force="--force" in sys.argv, verbose=True))
        print(build_capi_frame(verbose=True))
