"""Helper-wave A/B: one plan per case, solved with the helper wave off and on (interleaved
reps, HIP events), outputs compared bitwise between the two and, on a sample, with the oracle.

    python tools/helper_ab.py [cfg:n ...]        (default 2:4096 1:4096 3:4096)
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W  # noqa: E402
from many_bone_ik_amd.solver import Plan  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

dev = torch.device('cuda', 0)
cases = [(2, 4096), (1, 4096), (3, 4096)]
if len(sys.argv) > 1:
    cases = [tuple(int(x) for x in c.split(':')) for c in sys.argv[1:]]
st = torch.cuda.current_stream(dev).cuda_stream
for cfg, n in cases:
    wl = W.generate(cfg, n)
    p = Plan.from_workload(wl)
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    outs, times = {}, {0: [], 1: []}
    for rep in range(4):
        for h in (0, 1):
            p.set_helper_wave(h)
            po_ = torch.empty_like(pi)
            p.solve(pi.data_ptr(), tg.data_ptr(), po_.data_ptr(), 0, n, st)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                p.solve(pi.data_ptr(), tg.data_ptr(), po_.data_ptr(), 0, n, st)
            e1.record()
            torch.cuda.synchronize()
            times[h].append(e0.elapsed_time(e1) / 10)
            outs[h] = po_.cpu().numpy()
    same = np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    k = min(n, 64)
    idx = np.linspace(0, n - 1, k).astype(int)
    sub = W.generate(cfg, 1)
    ref_ok = True
    t0 = time.time()
    for i in idx[:16]:
        one = W.generate(cfg, 1, first=int(i))
        ref = po.Oracle(one).solve(one.pose, one.targets, threads=1)
        ref_ok &= np.array_equal(ref.view(np.uint32), outs[1][i:i + 1].view(np.uint32))
    print(json.dumps(dict(cfg=cfg, n=n, info={k2: p.info()[k2] for k2 in ("lanes_per_skeleton", "skeletons_per_block", "state_placement")},
                          off_ms=[round(x, 4) for x in times[0]], on_ms=[round(x, 4) for x in times[1]],
                          off_min=round(min(times[0]), 4), on_min=round(min(times[1]), 4),
                          bitwise_on_vs_off=bool(same), oracle16_bitwise=bool(ref_ok), oracle_s=round(time.time() - t0, 1))), flush=True)
    p.close()
