"""HIP path vs the oracle, through the C ABI (include/mbik.h).  Needs an MI355X: -m gpu.

Tolerance: the north star asks for bone quaternions within 1e-4 of the reference; the
HIP path reproduces the oracle's float rounding, so these tests assert bitwise equality
(which implies the 1e-4 bound) and report the max error when it fails."""
import glob
import os

import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, quat_error

pytestmark = pytest.mark.gpu
TOL = 1e-4


def assert_parity(got, ref, what=""):
    qe = quat_error(got, ref)
    assert np.isfinite(got).all(), what
    assert qe.max() <= TOL, f"{what}: max quaternion error {qe.max():.3e}"
    diff = np.argwhere(got.view(np.uint32) != ref.view(np.uint32))
    assert diff.size == 0, f"{what}: {len(diff)} values differ bitwise (max quat err {qe.max():.3e}); first {diff[:5].tolist()}"


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch, torch.device("cuda", 0)


@pytest.mark.parametrize("cfg,n", [(1, 4), (2, 96), (3, 96), (4, 24), (5, 6)])
@pytest.mark.parametrize("lanes", [0, 1, 4, 64])
def test_configs_bitwise_vs_oracle(oracle, mbik, cfg, n, lanes):
    wl = W.generate(cfg, n, first=1000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plan = Plan.from_workload(wl, lanes=lanes)
    assert_parity(plan.solve_host(wl.pose, wl.targets), ref, f"C{cfg} lanes={lanes}")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "oracle_c*.npz"))),
                         ids=os.path.basename)
def test_golden_fixtures(mbik, path):
    from tests.golden.make_golden import generate
    f = np.load(path, allow_pickle=False)
    wl = generate(f)
    plan = Plan.from_workload(wl)
    assert_parity(plan.solve_host(wl.pose, wl.targets), f["pose_out"], os.path.basename(path))
    r, t, _ = plan.segment_table()
    assert np.array_equal(r, f["seg_root"]) and np.array_equal(t, f["seg_tip"])


def test_c1_iteration_trace(oracle, mbik):
    """The reference's own CPU case (configs[0]): pose after every one of the 8 iterations."""
    wl = W.generate(1, 2)
    _, trace = oracle.Oracle(wl).solve(wl.pose, wl.targets, trace=True)
    for it in range(1, 9):
        plan = Plan.from_workload(wl, iterations=it)
        assert_parity(plan.solve_host(wl.pose, wl.targets), trace[:, it - 1], f"iteration {it}")
        plan.close()


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_segment_solve_vs_oracle(oracle, mbik, torch_dev, cfg):
    torch, dev = torch_dev
    wl = W.generate(cfg, 8)
    o = oracle.Oracle(wl)
    plan = Plan.from_workload(wl)
    nseg = plan.info()["segment_count"]
    for seg in sorted({0, nseg // 2, nseg - 1}):
        ref = o.segment_solve(seg, wl.pose, wl.targets)
        pose = torch.from_numpy(wl.pose.copy()).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        plan.segment_solve(seg, pose.data_ptr(), tg.data_ptr())
        torch.cuda.synchronize()
        assert_parity(pose.cpu().numpy(), ref, f"C{cfg} segment {seg}")


@pytest.mark.parametrize("cfg,n", [(2, 4096), (3, 65536)])
def test_full_size_properties(oracle, mbik, torch_dev, cfg, n):
    """BASELINE sizes: deterministic, finite, unit quaternions, slicing-invariant, and a random
    sub-sample bitwise equal to the oracle."""
    torch, dev = torch_dev
    wl = W.generate(cfg, n)
    plan = Plan.from_workload(wl)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    o1 = torch.empty_like(pi)
    o2 = torch.empty_like(pi)
    plan.solve(pi.data_ptr(), tg.data_ptr(), o1.data_ptr())
    plan.solve(pi.data_ptr(), tg.data_ptr(), o2.data_ptr())
    torch.cuda.synchronize()
    a, b = o1.cpu().numpy(), o2.cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "non-deterministic"
    assert np.isfinite(a).all()
    assert np.allclose(np.linalg.norm(a[..., :4].astype(np.float64), axis=-1), 1, atol=1e-5)
    # slice [first, first+count) of the batch == the same skeletons solved in the full batch
    first, count = n // 3, 257
    o3 = torch.empty((count,) + tuple(pi.shape[1:]), dtype=pi.dtype, device=dev)
    plan.solve(pi[first:].data_ptr(), tg[first:].data_ptr(), o3.data_ptr(), first, count)
    torch.cuda.synchronize()
    assert np.array_equal(o3.cpu().numpy().view(np.uint32), a[first:first + count].view(np.uint32))
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, 48, replace=False))
    for i in idx[:48]:
        sub = W.generate(cfg, 1, first=int(i))
        ref = oracle.Oracle(sub).solve(sub.pose, sub.targets)
        assert_parity(a[i:i + 1], ref, f"C{cfg} skeleton {i}")


def test_empty_and_invalid_ranges(mbik):
    wl = W.generate(3, 4)
    plan = Plan.from_workload(wl)
    out = plan.solve_host(wl.pose[:0], wl.targets[:0])
    assert out.shape[0] == 0
    with pytest.raises(_lib.MbikError) as e:
        plan.solve_host(wl.pose, wl.targets, first=2)  # 2 + 4 > 4
    assert e.value.code == _lib.MBIK_EINVAL
    with pytest.raises(_lib.MbikError):
        plan.set_launch(3)


def test_oversized_skeleton_fails_loudly(mbik):
    """A skeleton whose per-skeleton LDS state cannot fit one block is refused with
    MBIK_EUNSUPPORTED, never solved some other way."""
    B = 4000
    topo = W.custom_topology([-1] + list(range(B - 1)), [B - 1], [], iterations=1)
    wl = W.generate(3, 1, topo=topo)
    plan = Plan.from_workload(wl)
    with pytest.raises(_lib.MbikError) as e:
        plan.solve_host(wl.pose, wl.targets)
    assert e.value.code == _lib.MBIK_EUNSUPPORTED
    plan.close()
