"""Time mbik_solve under explicit layouts: args cfg:n:lanes:spw:interval[:placement:staging:waves[:roles]]
(0 = auto; placement / staging / waves / wave roles default to the plan's own).  Every layout's
output is compared bitwise with the first layout's of the same (cfg, n): `same` in the line."""
import sys, json
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan

dev = torch.device('cuda', 0)
cache = {}
first_out = {}
for arg in sys.argv[1:]:
    f = [int(x) for x in arg.split(':')]
    cfg, n, lanes, spw, interval = f[:5]
    if (cfg, n) not in cache:
        cache.clear()
        cache[(cfg, n)] = W.generate(cfg, n)
    wl = cache[(cfg, n)]
    p = Plan.from_workload(wl)
    p.set_layout(lanes, spw, interval)
    if len(f) > 5:
        p.set_locals_placement(f[5])
    if len(f) > 6:
        p.set_heading_staging(f[6])
    if len(f) > 7:
        p.set_waves_per_simd(f[7])
    if len(f) > 8:
        p.set_wave_roles(f[8])
    pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev); po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    inf = p.info()
    out = po.cpu()
    same = bool(torch.equal(out.view(torch.int32), first_out.setdefault((cfg, n), out).view(torch.int32)))
    print(json.dumps(dict(arg=arg, lanes=inf['lanes_per_skeleton'], spw=inf['skeletons_per_block'],
                          roles=inf.get('wave_roles', 0), wps=inf['waves_per_simd'], pl=inf['state_placement'],
                          lds=inf['lds_bytes_per_block'], ms=round(ms, 3), mskel_s=round(n / ms / 1e3, 3), same=same)), flush=True)
    p.close()
