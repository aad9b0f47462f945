"""A/B of solve-library variants on the GPU box: bitwise parity against the oracle on small
batches of C1-C5, then kernel time per config.  Each variant runs in its own process
(MBIK_LIB_OVERRIDE = build/abl/libmbik_abl_<tag>.so; BASE = whatever is named so too), and the
tags are interleaved over `--reps` rounds so that clock drift hits every variant alike.

    python tools/variant_check.py [--reps 2] [--cases 2:4096,3:65536] TAG [TAG ...]
A case is CFG:N (autotuned per variant) or CFG:N:K:spw:interval:staging:placement:waves[:helper]
(a pinned layout, as bench.py --layout).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(tag: str, cases: str, parity: bool):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from many_bone_ik_amd import workloads as W
    from many_bone_ik_amd.solver import Plan
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {"tag": tag}
    if parity:
        from oracle import pyoracle as po
        ok = {}
        for cfg, n in ((1, 1), (2, 48), (3, 48), (4, 16), (5, 8)):
            wl = W.generate(cfg, n, first=101)
            ref = po.Oracle(wl).solve(wl.pose, wl.targets, threads=16)
            p = Plan.from_workload(wl)
            got = p.solve_host(wl.pose, wl.targets)
            p.close()
            ok[f"c{cfg}"] = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
        out["bitwise"] = ok
    for case in cases.split(","):
        f = [int(x) for x in case.split(":")]
        cfg, n = f[:2]
        wl = W.generate(cfg, n)
        p = Plan.from_workload(wl)
        pi = torch.from_numpy(wl.pose).to(dev)
        tg = torch.from_numpy(wl.targets).to(dev)
        po_ = torch.empty_like(pi)
        if len(f) >= 8:
            # pinned layout CFG:N:K:spw:interval:staging:placement:waves[:helper[:roles]] (bench.py --layout)
            k, spw, interval, staging, placement, waves = f[2:8]
            p.set_helper_wave(f[8] if len(f) > 8 else 0)
            if hasattr(p._L, "mbik_plan_set_wave_roles"):
                p.set_wave_roles(f[9] if len(f) > 9 else 0)
            p.set_layout(k, spw, interval)
            p.set_heading_staging(staging)
            p.set_locals_placement(placement)
            p.set_waves_per_simd(waves)
        else:
            p.autotune(pi.data_ptr(), tg.data_ptr(), po_.data_ptr(), 0, n, st)
        for _ in range(2):
            p.solve(pi.data_ptr(), tg.data_ptr(), po_.data_ptr(), 0, n, st)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            p.solve(pi.data_ptr(), tg.data_ptr(), po_.data_ptr(), 0, n, st)
        e1.record()
        torch.cuda.synchronize()
        out[f"c{cfg}_ms" if len(f) < 8 else case] = round(e0.elapsed_time(e1) / reps, 4)
        p.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cases", default="2:4096")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--libdir", default=os.path.join("build", "abl"), help="where the variants' libraries are (build/abl is not pushed to GPU boxes)")
    a = ap.parse_args()
    if a.child:
        return child(a.tags[0], a.cases, not a.no_parity)
    for rep in range(a.reps):
        for tag in a.tags:
            env = dict(os.environ)
            env["MBIK_LIB_OVERRIDE"] = os.path.join(ROOT, a.libdir, f"libmbik_abl_{tag}.so")
            args = [sys.executable, os.path.abspath(__file__), "--child", tag, "--cases", a.cases]
            if a.no_parity or rep > 0:
                args.append("--no-parity")
            r = subprocess.run(args, env=env, timeout=600)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
