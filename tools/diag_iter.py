"""Per-iteration divergence of the HIP path vs the oracle trace."""
import sys
import numpy as np
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan, quat_error
from oracle import pyoracle as po

cfg = int(sys.argv[1]); n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wl = W.generate(cfg, n)
o = po.Oracle(wl)
ref, trace = o.solve(wl.pose, wl.targets, threads=8, trace=True)
for it in range(1, wl.topo.iterations + 1):
    p = Plan.from_workload(wl, iterations=it, lanes=1)
    out = p.solve_host(wl.pose, wl.targets)
    qe = quat_error(out, trace[:, it - 1])
    pe = np.abs(out[..., 4:7] - trace[:, it - 1, :, 4:7]).max(-1)
    worst = np.argsort(-qe.max(-1))[:2]
    print(f"iter {it}: max_qerr={qe.max():.3e} max_poserr={pe.max():.3e} nonzero_bones={int((qe>0).sum())}/{qe.size}", flush=True)
    if it <= 2:
        for s in worst:
            bones = np.nonzero(qe[s] > 0)[0]
            print(f"   skel {s}: bones with diff {bones.tolist()[:40]}  max {qe[s].max():.3e}")
    p.close()
