"""Solving-wave instruction accounting for helper-wave launches.

Needs the -DMBIK_REPLAY build (tools/replay_count.sh builds it and runs this under rocprofv3).
Per config: a helper-wave solve (mbik_solve_kernel_help), the same solve saving every helper
record (mbik_debug_replay mode 1), then the solving wave alone replaying those records
(mode 2, mbik_solve_kernel_replay: no partner, no waits).  The replay must reproduce the
helper launch bit for bit; its SQ counters are then the solving wave's own instruction stream.
    python tools/replay_count.py CFG:N [...]"""
import ctypes as C
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from many_bone_ik_amd import _lib, workloads as W  # noqa: E402
from many_bone_ik_amd.solver import Plan  # noqa: E402

dev = torch.device('cuda', 0)
L = _lib.load()
L.mbik_debug_replay.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
L.mbik_debug_replay.restype = C.c_int32
for case in sys.argv[1:]:
    cfg, n = (int(x) for x in case.split(':'))
    wl = W.generate(cfg, n)
    p = Plan.from_workload(wl)
    p.set_helper_wave(1)
    pi = torch.from_numpy(wl.pose).to(dev); tg = torch.from_numpy(wl.targets).to(dev)
    outs = [torch.empty_like(pi) for _ in range(3)]
    st = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(2):
        p.solve(pi.data_ptr(), tg.data_ptr(), outs[0].data_ptr(), 0, n, st.cuda_stream)
    ev[0].record(st)
    p.solve(pi.data_ptr(), tg.data_ptr(), outs[0].data_ptr(), 0, n, st.cuda_stream)
    ev[1].record(st)
    _lib.check(L.mbik_debug_replay(p.h, 1, 0, n, pi.data_ptr(), tg.data_ptr(), outs[1].data_ptr(), st.cuda_stream))
    ev[2].record(st)
    _lib.check(L.mbik_debug_replay(p.h, 2, 0, n, pi.data_ptr(), tg.data_ptr(), outs[2].data_ptr(), st.cuda_stream))
    ev[3].record(st)
    torch.cuda.synchronize()
    a, b, c = (o.cpu().numpy().view(np.uint32) for o in outs)
    print(json.dumps({"case": case, "helper_ms": ev[0].elapsed_time(ev[1]), "replay_ms": ev[2].elapsed_time(ev[3]),
                      "save_equal": bool(np.array_equal(a, b)), "replay_equal": bool(np.array_equal(a, c)),
                      "info": {k: p.info()[k] for k in ("lanes_per_skeleton", "skeletons_per_block", "helper_wave")}}), flush=True)
    _lib.check(L.mbik_debug_replay(p.h, 0, 0, 0, None, None, None, None))
    p.close()
