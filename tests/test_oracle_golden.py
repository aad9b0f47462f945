"""Oracle regression against the committed fixtures (tests/golden/make_golden.py) and the
generator's input digests."""
import glob
import os

import numpy as np
import pytest


FIX = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "oracle_c*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_generator_digest_stable(path):
    from tests.golden.make_golden import generate, input_digest
    f = load(path)
    wl = generate(f)
    assert input_digest(wl) == str(f["digest"])


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_oracle_reproduces_fixture(oracle, path):
    from tests.golden.make_golden import generate
    f = load(path)
    wl = generate(f)
    o = oracle.Oracle(wl)
    out, trace = o.solve(wl.pose, wl.targets, trace=True)
    assert np.array_equal(out.view(np.uint32), f["pose_out"].view(np.uint32))
    assert np.array_equal(trace[:, : f["trace"].shape[1]].view(np.uint32), f["trace"].view(np.uint32))
    assert o.bone_list() == f["bone_list"].tolist()
    r, t, nh = o.segment_table()
    assert np.array_equal(r, f["seg_root"]) and np.array_equal(t, f["seg_tip"]) and np.array_equal(nh, f["seg_nh"])
    seg0 = o.segment_solve(0, wl.pose, wl.targets)
    assert np.array_equal(seg0.view(np.uint32), f["segment0_pose"].view(np.uint32))


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_fixture_records_godot_version_and_oracle(path):
    """SURVEY §7 hard part 1 / §8(c): every fixture names the Godot-core version its arithmetic
    assumes and the oracle that produced it; the hash must be the current oracle's (an edited
    oracle means: rerun tests/golden/make_golden.py)."""
    from tests.golden.make_golden import GODOT_VERSION, oracle_source_hash
    f = load(path)
    assert str(f["godot_version"]) == GODOT_VERSION and str(f["godot_version"]).startswith("4.3")
    assert str(f["oracle_sha256"]) == oracle_source_hash(), "oracle sources changed since the fixture was made"
    assert "glibc 2.35" in str(f["libm"])
