import sys, numpy as np
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, quat_error
from oracle import pyoracle as po
for (cfg, n, k, wps, it) in [(2, 70, 8, 2, 16), (2, 70, 8, 2, 1), (2, 64, 8, 2, 1), (2, 6, 8, 2, 1), (2, 70, 4, 2, 1)]:
    wl = W.generate(cfg, n, first=51000 + cfg)
    ref = po.Oracle(wl, iterations=it).solve(wl.pose, wl.targets, threads=8)
    p = Plan.from_workload(wl, iterations=it)
    p.set_layout(k, 0, 0); p.set_waves_per_simd(wps); p.set_wave_roles(1)
    got = p.solve_host(wl.pose, wl.targets)
    qe = quat_error(got, ref)
    bad_sk = np.where(qe.max(axis=1) > 0)[0]
    bad_b = np.where(qe.max(axis=0) > 0)[0]
    neq = (got.view(np.uint32) != ref.view(np.uint32))
    print(cfg, n, k, wps, it, "maxerr", qe.max(), "bad skeletons", bad_sk[:20].tolist(), len(bad_sk), "bad bones", bad_b.tolist(), "neq", int(neq.sum()), flush=True)
