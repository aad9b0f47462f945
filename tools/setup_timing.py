"""Host plan creation vs GPU setup rebuild (mbik_plan_rebuild_setup) per config."""
import json, sys, time
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

dev = torch.device('cuda', 0)
torch.zeros(1, device=dev)
for cfg, n in ((2, 4096), (3, 65536), (4, 32768), (5, 16384)):
    wl = W.generate(cfg, n)
    t0 = time.perf_counter(); p = Plan.from_workload(wl); t1 = time.perf_counter()
    pose, cones, twist = (torch.from_numpy(a).to(dev) for a in (wl.pose, wl.cones, wl.twist))
    st = torch.cuda.current_stream().cuda_stream
    p.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=st)
    torch.cuda.synchronize()
    reps = 3
    t2 = time.perf_counter()
    for _ in range(reps):
        p.rebuild_setup(pose.data_ptr(), cones.data_ptr(), twist.data_ptr(), stream=st)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(json.dumps(dict(cfg=cfg, n=n, host_plan_create_ms=round((t1 - t0) * 1e3, 1),
                          gpu_setup_rebuild_ms=round((t3 - t2) / reps * 1e3, 2))), flush=True)
