"""Per-phase cycle accounting of the solve kernel (needs a -DMBIK_PROF build named by
MBIK_LIB_OVERRIDE, see tools/prof_build.sh).  Prints, per config, the share of wave
cycles spent in each phase (summed over waves; one solve launch)."""
import ctypes as C, json, os, sys
import torch
sys.path.insert(0, '.')
from many_bone_ik_amd import _lib, workloads as W
from many_bone_ik_amd.solver import Plan

NAMES = ["load", "headings_qcp", "clamp_slerp_rotate", "swing", "twist", "global_pass", "store", "total",
         "step_start", "eff_headings", "qcp_adjugate", "convert_clamp", "slerp", "translate_steps", "qcp_centroid_sums", "tr_headings_build", "tr_staged_sums", "tr_rotate", "help_wait", "help_wait_b", "help_wait_first", "helper_global_pass", "helper_first_record"]
# wave roles (ROLES=1): counters 18-23 are the cooperative rows' (solve_block.h)
NAMES_RW = NAMES[:18] + ["rw_plain_rows", "rw_coop_walk", "rw_coop_sums", "rw_coop_barrier_wait", "rw_coop_steps", "rw_coop_rows"]
dev = torch.device('cuda', 0)
L = _lib.load()
L.mbik_debug_prof.argtypes = [C.c_void_p]
buf = (C.c_ulonglong * 24)()
for case in sys.argv[1:]:
    # CFG:N:LANES[:SPW:INTERVAL[:STAGING:PLACEMENT:WAVES[:ROLES]]]
    parts = [int(x) for x in case.split(':')]
    cfg, n, lanes = parts[:3]
    spw, interval = (parts[3:5] + [0, 0])[:2] if len(parts) > 3 else (0, 0)
    wl = W.generate(cfg, n)
    p = Plan.from_workload(wl, lanes=lanes)
    if spw or interval:
        p.set_layout(lanes, spw, interval)
    if len(parts) > 5:
        staging, placement, waves = parts[5:8]
        p.set_heading_staging(staging)
        p.set_locals_placement(placement)
        p.set_waves_per_simd(waves)
    if os.environ.get("MBIK_HELP"):
        p.set_helper_wave(int(os.environ["MBIK_HELP"]))
    rw = len(parts) > 8 and parts[8] == 1
    if rw:
        p.set_wave_roles(1)
    pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev); po = torch.empty_like(pi)
    st = torch.cuda.current_stream(dev).cuda_stream
    p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st); torch.cuda.synchronize()
    L.mbik_debug_prof(buf)
    p.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), 0, n, st); torch.cuda.synchronize()
    L.mbik_debug_prof(buf)
    v = list(buf)
    inf = p.info()
    waves = (n + inf['skeletons_per_block'] - 1) // inf['skeletons_per_block']
    if inf.get('wave_roles'):
        waves *= inf['lanes_per_skeleton']             # K waves per block
    out = dict(cfg=cfg, n=n, lanes=inf['lanes_per_skeleton'], spw=inf['skeletons_per_block'], case=case,
               cycles_per_wave=round(v[7] / waves))
    out.update({k: round(x / max(1, v[7]), 4) for k, x in zip(NAMES_RW if inf.get('wave_roles') else NAMES, v) if k != "total"})
    print(json.dumps(out), flush=True)
    p.close()
