"""constraint_mode layout probe: ms per frame of pinned layouts on one batch, each timed from the
same saved node caches (a fresh plan per layout, two warm-up frames, then the mean of five).
python tools/cmode_probe.py CFG:N lanes:spw:roles [...]"""
import json, sys
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

dev = torch.device('cuda', 0)
cfg, n = (int(x) for x in sys.argv[1].split(':'))
wl = W.generate(cfg, n)
pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev); po = torch.empty_like(pi)
st = torch.cuda.current_stream(dev).cuda_stream
for spec in sys.argv[2:]:
    lanes, spw, roles = (int(x) for x in spec.split(':'))
    p = Plan.from_workload(wl, constraint_mode=True, lanes=lanes)
    p.set_wave_roles(roles)
    p.set_layout(lanes, spw, 0)
    for _ in range(2):
        p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    e1.record(); torch.cuda.synchronize()
    inf = p.info()
    print(json.dumps(dict(cfg=cfg, n=n, spec=spec, ms=round(e0.elapsed_time(e1) / 5, 3), lanes=inf["lanes_per_skeleton"],
                          spb=inf["skeletons_per_block"], rw=inf["wave_roles"], lds=inf["lds_bytes_per_block"])), flush=True)
    p.close()
