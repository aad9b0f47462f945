"""Debug one fuzz case: find the first iteration / lane count where GPU and oracle differ."""
import sys
import numpy as np
sys.path.insert(0, '.')
from tests.test_gpu_fuzz import random_case
from many_bone_ik_amd.solver import Plan, quat_error
from oracle import pyoracle as po

seed = int(sys.argv[1])
wl, stab, lanes = random_case(seed)
for ln in (0, 1, 4, 64):
    for it in range(1, wl.topo.iterations + 1):
        ref = po.Oracle(wl, stabilization_passes=stab, iterations=it).solve(wl.pose, wl.targets)
        got = Plan.from_workload(wl, lanes=ln, stabilization_passes=stab, iterations=it).solve_host(wl.pose, wl.targets)
        d = np.argwhere(got.view(np.uint32) != ref.view(np.uint32))
        if d.size:
            print(f"lanes={ln} first diff at iteration {it}: {len(d)} values; skeletons {sorted(set(d[:,0].tolist()))[:8]} bones {sorted(set(d[:,1].tolist()))}")
            s, b = d[0, 0], d[0, 1]
            print('  got', got[s, b], '\n  ref', ref[s, b])
            break
    else:
        print(f"lanes={ln}: bitwise equal for all iterations")
