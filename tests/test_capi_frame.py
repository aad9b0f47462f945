"""The boundary proven from C: tests/capi_frame.c, a C99 program that includes
only include/mbik.h and links libmbik.so, runs INTEGRATION.md §3's frame loop --
mbik_plan_create -> per frame mbik_capture_targets -> mbik_solve_checked -> read back, the output
pose feeding the next frame (many_bone_ik_3d.cpp:91-116, :645-694) -- and every frame's captured
targets and poses are compared bitwise with the oracle.

The compile check (gcc -std=c99 -Wall -Wextra -Werror against the header) runs without a GPU;
the frame loop needs an MI355X: -m gpu."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from many_bone_ik_amd import build as B
from many_bone_ik_amd import workloads as W

from .test_gpu_capture import random_xforms
from .test_gpu_parity import assert_parity


def test_capi_frame_compiles_as_c99(mbik):
    """A C caller that reads only the header compiles warning-free and links (no GPU)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "capi_frame")
        subprocess.run(B.capi_frame_cmd(out), check=True)
        env = dict(os.environ, LD_LIBRARY_PATH=B.HERE)      # (the $ORIGIN rpath points elsewhere from here)
        r = subprocess.run([out], capture_output=True, text=True, timeout=60, env=env)
        assert r.returncode == 1 and "usage" in r.stderr


def write_input(path, wl, skel_global, target_global, shards=0):
    t = wl.topo
    P, C = t.pins.shape[0], t.constrained.shape[0]
    MC = wl.cones.shape[2]
    frames = target_global.shape[0]
    with open(path, "wb") as f:
        np.array([wl.bone_count, P, C, MC, t.iterations, wl.n, frames, shards], np.int32).tofile(f)
        t.parents.astype(np.int32).tofile(f)
        t.pins.astype(np.int32).tofile(f)
        wl.pin_weight.astype(np.float32).tofile(f)
        wl.pin_priority.astype(np.float32).tofile(f)
        wl.pin_propagation.astype(np.float32).tofile(f)
        t.constrained.astype(np.int32).tofile(f)
        wl.cone_count.astype(np.int32).tofile(f)
        np.array([wl.default_damp], np.float32).tofile(f)
        for a in (wl.pose, wl.cones, wl.twist, skel_global, target_global):
            np.ascontiguousarray(a, np.float32).tofile(f)


def read_output(path, wl, frames, shards=0):
    n, Bn, P = wl.n, wl.bone_count, wl.topo.pins.shape[0]
    raw = np.fromfile(path, np.uint8)
    per = n * P * 12 * 4 + n * Bn * 10 * 4 + n
    multi = n * Bn * 40 if shards else 0
    assert raw.size == frames * per + multi, (raw.size, frames * per + multi)
    out = []
    for f in range(frames):
        r = raw[f * per:(f + 1) * per]
        tg = r[:n * P * 48].view(np.float32).reshape(n, P, 12)
        pose = r[n * P * 48:n * P * 48 + n * Bn * 40].view(np.float32).reshape(n, Bn, 10)
        nf = r[n * P * 48 + n * Bn * 40:]
        out.append((tg, pose, nf))
    if shards:
        out.append(raw[frames * per:].view(np.float32).reshape(n, Bn, 10))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,rest,shards", [(2, 256, "plus_y", 3), (2, 128, "realistic", 2), (4, 32, "realistic", 0)])
def test_c_frame_loop_bitwise_vs_oracle(oracle, mbik, cfg, n, rest, shards):
    """shards > 0: frame 0 once more through mbik_multi_create / mbik_multi_solve over that many
    plans (the single-process multi-GPU entry points), equal to frame 0."""
    exe = B.CAPI_FRAME
    assert os.path.exists(exe), "tests/capi_frame not built: __graft_entry__.build() builds it"
    wl = W.generate(cfg, n, first=5000, rest=rest)
    rng = np.random.default_rng(cfg * 31 + n)
    frames = 3
    P = wl.topo.pins.shape[0]
    skel = random_xforms(rng, (n,))                       # scene-space skeleton transforms, scaled
    # scene-space target nodes: the synthetic targets carried into the scene, drifting per frame
    tgl = np.empty((frames, n, P, 12), np.float32)
    for f in range(frames):
        drift = wl.targets.copy()
        drift[..., 9:12] += np.float32(0.05 * f) * rng.standard_normal((n, P, 3)).astype(np.float32)
        for s in range(n):
            for e in range(P):
                tgl[f, s, e] = oracle.xform_mul(skel[s], drift[s, e])
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        write_input(fin, wl, skel, tgl, shards)
        r = subprocess.run([exe, fin, fout], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr + r.stdout
        got = read_output(fout, wl, frames, shards)
    multi = got.pop() if shards else None
    o = oracle.Oracle(wl)
    pose = wl.pose
    for f, (tg, out, nf) in enumerate(got):
        want_tg = np.stack([np.stack([oracle.xform_mul(oracle.xform_affine_inverse(skel[s]), tgl[f, s, e])
                                      for e in range(P)]) for s in range(n)])
        assert np.array_equal(tg.view(np.uint32), want_tg.view(np.uint32)), f"frame {f}: captured targets differ"
        ref = o.solve(pose, want_tg, threads=8)
        assert_parity(out, ref, f"C frame loop, {rest} C{cfg}, frame {f}")
        assert not nf.any()
        if f == 0 and multi is not None:
            assert_parity(multi, ref, f"C mbik_multi_solve over {shards} plans, {rest} C{cfg}")
        pose = ref
