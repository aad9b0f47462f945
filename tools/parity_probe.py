"""Quick parity probe: HIP path vs oracle on small batches of every config."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, quat_error
from oracle import pyoracle as po

for cfg in [int(c) for c in (sys.argv[1:] or ['1', '3', '2', '4', '5'])]:
    n = {1: 4, 2: 64, 3: 64, 4: 32, 5: 8}[cfg]
    wl = W.generate(cfg, n)
    o = po.Oracle(wl)
    ref = o.solve(wl.pose, wl.targets, threads=8)
    for lanes in [0, 64, 1]:
        p = Plan.from_workload(wl, lanes=lanes)
        t0 = time.time(); out = p.solve_host(wl.pose, wl.targets); dt = time.time() - t0
        qe = quat_error(out, ref)
        pe = np.abs(out[..., 4:7] - ref[..., 4:7]).max()
        frac = np.mean(qe.max(-1) <= 1e-4)
        print(f"cfg{cfg} lanes={lanes} info={ {k: v for k, v in p.info().items() if k in ('lanes_per_skeleton','skeletons_per_block','segment_count','level_count')} } "
              f"max_qerr={qe.max():.3e} frac<=1e-4={frac:.3f} max_poserr={pe:.3e} finite={np.isfinite(out).all()} t={dt*1e3:.1f}ms", flush=True)
        p.close()
