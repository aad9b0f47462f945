"""Synthetic generator: counts, determinism, per-skeleton streams."""
import numpy as np
import pytest

from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import describe_topology

# (bones, effectors, segments, headings of the root segment) per config
EXPECT = {1: (8, 1, 1, 5), 2: (32, 4, 5, 20), 3: (32, 4, 5, 20), 4: (64, 8, 11, 40), 5: (200, 16, 21, 80)}


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_topology_counts(mbik, cfg):
    t = W.topology(cfg)
    B, P, S, H = EXPECT[cfg]
    assert t.parents.shape[0] == B and t.pins.shape[0] == P
    d = describe_topology(t.parents, [dict(bone=int(b), weight=1.0) for b in t.pins])
    assert len(d["seg_root"]) == S
    assert d["seg_headings"][-1] == H          # post-order: the root segment comes last
    assert sorted(d["bone_list"].tolist()) == list(range(B))


@pytest.mark.parametrize("cfg", [2, 5])
def test_slices_regenerate_identically(cfg):
    a = W.generate(cfg, 6)
    b = W.generate(cfg, 3, first=2)
    for x, y in [(a.pose[2:5], b.pose), (a.targets[2:5], b.targets), (a.cones[2:5], b.cones)]:
        assert np.array_equal(x, y)


def test_inputs_are_sane():
    wl = W.generate(2, 16)
    q = wl.pose[..., :4].astype(np.float64)
    assert np.allclose(np.linalg.norm(q, axis=-1), 1, atol=1e-6)
    assert np.all(wl.pose[..., 7:10] == 1)
    assert np.allclose(np.linalg.norm(wl.cones[..., :3], axis=-1), 1, atol=1e-5)
    assert np.all((wl.pose[:, 1:, 5] >= 0.8) & (wl.pose[:, 1:, 5] <= 1.2))
    R = wl.targets[..., :9].reshape(16, 4, 3, 3).astype(np.float64)
    assert np.allclose(R @ np.swapaxes(R, -1, -2), np.eye(3), atol=1e-5)


def test_c5_finger_lengths():
    t = W.topology(5)
    kids = np.bincount(t.parents[t.parents >= 0], minlength=200)
    assert (kids == 0).sum() == 16 and t.parents.shape[0] == 200
