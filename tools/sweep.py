"""Time mbik_solve for several configs / lane counts (no parity, no CPU baseline)."""
import sys, time, json
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

dev = torch.device('cuda', 0)
cases = [(2, 4096), (3, 65536), (5, 16384), (4, 32768)]
if len(sys.argv) > 1:
    cases = [tuple(int(x) for x in c.split(':')) for c in sys.argv[1:]]
for case in cases:
    cfg, n = case[0], case[1]
    wl = W.generate(cfg, n)
    for lanes in (case[2:] or [0, 4, 8, 16, 32, 64]):
        try:
            p = Plan.from_workload(wl, lanes=lanes)
        except Exception as e:
            print(cfg, n, lanes, 'ERR', e, flush=True); continue
        inf = p.info()
        pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev); po = torch.empty_like(pi)
        st = torch.cuda.current_stream(dev).cuda_stream
        try:
            p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st); torch.cuda.synchronize()
        except Exception as e:
            print(cfg, n, lanes, 'ERR', e, flush=True); p.close(); continue
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record()
        for _ in range(reps):
            p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        inf = p.info()
        print(json.dumps(dict(cfg=cfg, n=n, lanes=inf["lanes_per_skeleton"], spw=inf["skeletons_per_block"], lds=inf["lds_bytes_per_block"], ms=round(ms, 3),
                              mskel_s=round(n / ms / 1e3, 3))), flush=True)
        p.close()
