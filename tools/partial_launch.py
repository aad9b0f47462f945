"""Launch time against batch size on one autotuned plan (chunked mbik_solve_host).

A fully resident launch is as long as one skeleton's serial chain, so a launch of a quarter of
the batch should take about as long as the whole batch, and k chunks solved one after another
about k times as long. This times plan.solve over the first n skeletons, and k back-to-back
chunks of n/k, on the plan autotune picked for the whole batch.

  python tools/partial_launch.py [--config 2] [--n 4096] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from many_bone_ik_amd import workloads as W  # noqa: E402
from many_bone_ik_amd.solver import Plan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.generate(a.config, a.n)
    plan = Plan.from_workload(wl, device=0)
    pin = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    out = torch.empty_like(pin)
    s = torch.cuda.current_stream(dev).cuda_stream
    plan.autotune(pin.data_ptr(), tg.data_ptr(), out.data_ptr(), 0, a.n, s)

    def timed(chunks):
        for _ in range(3):
            for f, c in chunks:
                plan.solve(pin.data_ptr(), tg.data_ptr(), out.data_ptr(), f, c, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record()
        for _ in range(a.reps):
            for f, c in chunks:
                plan.solve(pin.data_ptr(), tg.data_ptr(), out.data_ptr(), f, c, s)
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / a.reps

    rows = []
    for frac in (1, 2, 4, 8, 16):
        n = a.n // frac
        rows.append({"kind": "first_n", "skeletons": n, "ms": timed([(0, n)])})
    for k in (2, 4, 8):
        c = a.n // k
        rows.append({"kind": "chunks_in_series", "chunks": k, "skeletons": a.n,
                     "ms": timed([(i * c, c) for i in range(k)])})
    info = plan.info()
    for r in rows:
        r.update(config=a.config, batch=a.n, lanes=info.get("lanes_per_skeleton"),
                 skeletons_per_block=info.get("skeletons_per_block"), helper_wave=info.get("helper_wave"),
                 state_placement=info.get("state_placement"))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
