"""Per-phase accounting of the constraint_mode kernel (a -DMBIK_PROF build named by
MBIK_LIB_OVERRIDE): cycles per lane in each phase of cmode_step, and how much dirty-chain
recomputation a frame does.  python tools/prof_cmode.py CFG:N [...]"""
import ctypes as C, json, sys
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import _lib, workloads as W
from many_bone_ik_amd.solver import Plan

NAMES = {0: "eff_heading_reads", 1: "swing", 2: "twist", 4: "dirty_chain_cycles", 8: "row_cleaning"}
dev = torch.device('cuda', 0)
L = _lib.load()
L.mbik_debug_prof.argtypes = [C.c_void_p]
buf = (C.c_ulonglong * 24)()
for case in sys.argv[1:]:
    # CFG:N (autotuned layout) or CFG:N:lanes:spw:roles (pinned)
    f = [int(x) for x in case.split(':')]
    cfg, n = f[:2]
    wl = W.generate(cfg, n)
    p = Plan.from_workload(wl, constraint_mode=True, lanes=f[2] if len(f) > 2 else 0)
    pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev); po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    if len(f) > 2:
        p.set_wave_roles(f[4])
        p.set_layout(f[2], f[3], 0)
    else:
        p.autotune(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)  # the bench's layout
    p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st); torch.cuda.synchronize()
    L.mbik_debug_prof(buf)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st)
    e1.record(); torch.cuda.synchronize()
    L.mbik_debug_prof(buf)
    v = list(buf)
    lanes = n * p.info()["lanes_per_skeleton"]
    out = dict(cfg=cfg, n=n, ms=round(e0.elapsed_time(e1), 3), lanes=p.info()["lanes_per_skeleton"], spb=p.info().get("skeletons_per_block"), rw=p.info()["wave_roles"],
               cycles_per_lane=round(v[7] / lanes))
    out.update({nm: round(v[i] / max(1, v[7]), 4) for i, nm in NAMES.items()})
    out.update(chain_nodes_per_skeleton=round(v[5] / n), dirty_pose_reads_per_skeleton=round(v[6] / n),
               bdir_recomputes_per_skeleton=round(v[9] / n), private_nodes_per_skeleton=round(v[10] / n),
               group_chain_nodes_per_skeleton=round(v[11] / n), group_step_cycles=round(v[12] / max(1, v[7]), 4),
               multi_effector_step_cycles=round(v[13] / max(1, v[7]), 4))
    print(json.dumps(out), flush=True)
    p.close()
