"""Multi-GPU in the library: mbik_multi_create / mbik_multi_solve shard one
batch over several plans -- contiguous skeleton ranges, each plan on its own device and a stream
the handle owns -- and gather the poses to the root device (the per-frame call is
many_bone_ik_3d.cpp:645-694).  On the one-GPU box the plans share device 0: without staging the
shards solve in place on concurrent streams, and MBIK_MULTI_STAGE_ALL runs the scatter / solve /
gather copy path that separate devices use.  Bitwise against the oracle.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from many_bone_ik_amd import _lib
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Multi, Plan

from .test_gpu_parity import assert_parity, torch_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def shard_plans(wl, cuts, **kw):
    """One plan per contiguous range [cuts[i], cuts[i+1]) of the workload's skeletons."""
    return [Plan(wl.topo.parents, wl.pins(), wl.constraints(), wl.pose[lo:hi], wl.cones[lo:hi], wl.twist[lo:hi],
                 iterations=wl.topo.iterations, default_damp=wl.default_damp, max_cones=wl.cones.shape[2], **kw)
            for lo, hi in zip(cuts[:-1], cuts[1:])]


@pytest.mark.parametrize("cfg,n,cuts", [(2, 300, [0, 100, 300]), (4, 130, [0, 64, 65, 130]), (5, 40, [0, 13, 26, 40])])
@pytest.mark.parametrize("stage_all", [False, True])
def test_multi_solve_bitwise_vs_oracle(oracle, mbik, torch_dev, cfg, n, cuts, stage_all):
    torch, dev = torch_dev
    wl = W.generate(cfg, n, first=61000 + cfg)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    plans = shard_plans(wl, cuts)
    m = Multi(plans, root_device=0, stage_all=stage_all)
    assert m.skeletons() == (n, cuts)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    po = torch.full_like(pi, float("nan"))
    st = torch.cuda.Stream(dev)
    for _ in range(2):                   # twice: the handle's streams and events are reused
        m.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), st.cuda_stream)
        st.synchronize()
        assert_parity(po.cpu().numpy(), ref, f"C{cfg} multi over {len(plans)} plans stage_all={stage_all}")


def test_multi_in_place_and_stream_order(oracle, mbik, torch_dev):
    """pose_out == pose_in, with work queued on the root stream before and after the call."""
    torch, dev = torch_dev
    wl = W.generate(2, 200, first=62000)
    ref = oracle.Oracle(wl).solve(wl.pose, wl.targets, threads=8)
    m = Multi(shard_plans(wl, [0, 77, 200]), stage_all=True)
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        pose = torch.zeros(wl.pose.shape, dtype=torch.float32, device=dev)
        pose.copy_(torch.from_numpy(wl.pose).to(dev, non_blocking=True))       # queued before the solve
        tg = torch.from_numpy(wl.targets).to(dev)
        m.solve(pose.data_ptr(), tg.data_ptr(), pose.data_ptr(), st.cuda_stream)
        after = pose.clone()                                                   # queued after it
    st.synchronize()
    assert_parity(after.cpu().numpy(), ref, "multi in place")


def test_multi_argument_checks(mbik):
    a = Plan.from_workload(W.generate(2, 8))
    b = Plan.from_workload(W.generate(3, 8))
    c = Plan.from_workload(W.generate(4, 8))              # 64 bones: not the same shape
    for plans, root in ([a, a], 0), ([a, c], 0), ([a, b], 99):
        with pytest.raises(_lib.MbikError) as e:
            Multi(plans, root_device=root)
        assert e.value.code == _lib.MBIK_EINVAL
    m = Multi([a, b])
    assert m.skeletons() == (16, [0, 8, 16])
    with pytest.raises(_lib.MbikError):
        m.solve(0, 0, 0)


def test_bench_library_multi_on_one_box(mbik, torch_dev):
    """bench.py's library_multi measurement: at N > 1 rank 0 times
    mbik_multi_solve over one plan per visible device while the other ranks wait.  The same
    code on the one-GPU box, with both plans on device 0, run as the driver runs bench.py:
    the line carries the measurement and its oracle checks at both ends of the batch."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--config", "2", "--skeletons", "256", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-autotune", "--pmc", "off", "--library-multi-devices", "0,0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    lm = line["library_multi"]
    assert "error" not in lm, lm
    assert lm["devices"] == [0, 0] and lm["plans"] == 2 and lm["skeletons"] == 256 and lm["ms_per_frame"] > 0
    assert [c["range"] for c in lm["parity"]] == [[0, 16], [240, 256]]
    assert all(c["bitwise_equal"] for c in lm["parity"]), lm["parity"]
    # the line's own parity check covers both ends of the rank's batch as well
    assert line["parity"]["ranges"] == [[0, 32], [224, 256]] and line["parity"]["bitwise_equal"]
