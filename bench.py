#!/usr/bin/env python3
"""Benchmark: skeletons/s solved to convergence (fixed 16 iterations) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]

One *step* = one mbik_solve() over this rank's batch of skeletons (BASELINE.json
configs[1] = C2 by default: 4096 x 32 bones / 4 effectors / 2 Kusudama cones per bone,
16 iterations), inputs already resident in HBM.  Rank 0 prints one JSON line.

N > 1 runs one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is
a rank; WORLD_SIZE must equal --gpus.  Run as a plain command with --gpus N > 1, it starts
torch.distributed.run itself as a child process (before anything touches the GPU) and exits
with its status.  Every rank solves its own contiguous shard of skeletons with no
collective on the data path:
  --scaling weak    (default) the config's skeletons_per_gpu on every rank;
  --scaling strong  the config's whole batch (C4: 262,144) split by dist.shard_range.
The RCCL gathers of the output poses are timed separately after the solve loop.  At N > 1
rank 0 then also times the library's own multi-GPU path (mbik_multi_solve: one process, one
plan per visible device, peer-copy scatter / gather to device 0) over the whole batch while the
other ranks wait on the host; it is reported under "library_multi", never as `value`.
(--library-multi-devices 0,0 runs that measurement at N = 1 with the listed devices' plans:
the one-GPU test of the same code.)

At N = 1, after the timed region, rank 0 re-runs the timed layout in rocprofv3 --pmc child
processes (FETCH_SIZE, WRITE_SIZE, SQ wave counters; `--pmc off` skips them): the line's
roofline.traffic and pmc_live.per_wave come from this run, not from committed files.

--dry-run exercises the launcher / rendezvous / sharding / timing plumbing on CPU (gloo,
no GPU, no solve): the tests use it, its line says "dry_run": true and is never a result.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
VALU_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (same guide)
SKEL_PER_GPU = {2: 4096, 3: 65536, 4: 262144 // 8, 5: 16384}      # weak scaling
SKEL_TOTAL = {2: 4096, 3: 65536, 4: 262144, 5: 16384}             # strong scaling (BASELINE configs)
METRIC = "skeletons/sec to convergence (32-bone/4-eff, 16 iters) at 1/2/4/8 GPU; bone-quat max-err vs ref"


def progress(msg: str) -> None:
    """One line per phase on stderr: long runs (262,144-skeleton batches, autotune) keep writing."""
    print(f"[bench {time.strftime('%H:%M:%S')} rank {os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--skeletons", type=int, default=0,
                    help="skeletons per GPU (weak) or in total (strong); default: the config's")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only plumbing check: gloo, no GPU, no solve (tests)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per skeleton override (0 = plan default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-autotune", action="store_true", help="keep the plan's automatic launch layout")
    ap.add_argument("--layout", default="",
                    help="pin a launch layout instead of autotuning: K:spw:interval:staging:placement:waves[:helper[:wave_roles]] "
                         "(mbik_plan_info's fields; tools/round_profile.sh passes the one its first run picked)")
    ap.add_argument("--constraint-mode", action="store_true",
                    help="ManyBoneIK3D::constraint_mode (snaps only; each step is one frame of the persistent node caches)")
    ap.add_argument("--stabilization-passes", type=int, default=0)
    ap.add_argument("--library-multi-devices", default="",
                    help="comma-separated devices for the library_multi measurement (default at N > 1: 0..N-1)")
    ap.add_argument("--pmc", choices=["auto", "on", "off", "child"], default=os.environ.get("MBIK_BENCH_PMC", "auto"),
                    help="measure roofline.traffic and the VALU issue of the timed layout in this run with rocprofv3 "
                         "--pmc children (auto: at N=1 when rocprofv3 is present and this run is not itself profiled)")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "traffic.json"))
    ap.add_argument("--valu-mix-json", default=os.path.join(HERE, "profiles", "valu_mix.json"))
    return ap.parse_args()


def host_cpu() -> dict:
    """The host cores this process may run on: affinity (what `nproc` prints), the cgroup CPU
    quota if one is set, os.cpu_count() (the whole machine) and the CPU model."""
    info = {"nproc": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "cgroup_quota_cpus": None,
            "cpu_model": None}
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def cpu_baseline(cfg: int, seconds: float, **flags):
    """Oracle (plain-C restatement of the reference) on every host core this process may use
    (`nproc` threads), bounded sample of the same workload."""
    from many_bone_ik_amd import workloads as W
    from oracle import pyoracle as po
    hc = host_cpu()
    # every core this process may use: the affinity set (`nproc`), capped by the cgroup CPU
    # quota when one is set -- on the GPU box the affinity set is the whole 256-thread machine
    # but the quota is 16 CPUs, and 256 threads on 16 CPUs only get throttled (31.5 k vs 37.8 k
    # skeletons/s measured)
    threads = hc["nproc"] if not hc["cgroup_quota_cpus"] else max(1, min(hc["nproc"], math.ceil(hc["cgroup_quota_cpus"])))
    n = max(512, 8 * threads) if cfg in (2, 3, 4) else max(64, 2 * threads)
    wl = W.generate(cfg, n)
    o = po.Oracle(wl, **flags)
    done = 0
    t0 = time.perf_counter()
    while True:
        o.solve(wl.pose, wl.targets, threads=threads)
        done += n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    o.close()
    return {"value": done / el, "unit": "skeletons/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ (C restatement of the reference solve, platform libm) on config C{cfg}: "
                      f"{n} skeletons solved {done // n} times in {el:.1f} s with {threads} threads",
            **hc}


def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) run as a plain command: start torch.distributed.run with N
    ranks as a child process and return its exit status (non-zero if any rank failed).  This
    parent never imports torch or touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)



def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a 1-GPU box (never set by the driver): every rank on one device, and
    # the process-group backend ("nccl" = RCCL by default; "gloo" carries device tensors too).
    if os.environ.get("MBIK_BENCH_DEVICE"):
        local_rank = int(os.environ["MBIK_BENCH_DEVICE"])
    backend = os.environ.get("MBIK_BENCH_BACKEND", "nccl")
    if world != args.gpus:
        sys.exit(f"WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU is required")
    if args.dry_run:
        return dry_run(args, world, rank)
    dist = None
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        # a host-only group: the other ranks wait on it while rank 0 drives every GPU (library_multi)
        host_group = dist.new_group(backend="gloo")
    dev = torch.device("cuda", local_rank)

    from many_bone_ik_amd import workloads as W
    from many_bone_ik_amd.solver import Plan, quat_error

    cfg = args.config
    total, first, n = batch_shard(args, world, rank)
    progress(f"generate C{cfg}: {n} skeletons from {first}")
    wl = W.generate(cfg, n, first=first)
    flags = dict(constraint_mode=args.constraint_mode, stabilization_passes=args.stabilization_passes)
    progress("plan")
    plan = Plan.from_workload(wl, device=local_rank, lanes=args.lanes, **flags)
    info = plan.info()
    pose_in = torch.from_numpy(wl.pose).to(dev)
    targets = torch.from_numpy(wl.targets).to(dev)
    pose_out = torch.empty_like(pose_in)
    stream = torch.cuda.current_stream(dev)

    def step():
        plan.solve(pose_in.data_ptr(), targets.data_ptr(), pose_out.data_ptr(), 0, n, stream.cuda_stream)

    if args.layout:
        fields = [int(x) for x in args.layout.split(":")]
        k, spw, interval, staging, placement, waves = fields[:6]
        plan.set_helper_wave(fields[6] if len(fields) > 6 else 0)
        plan.set_wave_roles(fields[7] if len(fields) > 7 else 0)
        plan.set_layout(k, spw, interval)
        plan.set_heading_staging(staging)
        plan.set_locals_placement(placement)
        plan.set_waves_per_simd(waves)
        step()
        info = plan.info()
    elif not args.no_autotune:
        # mbik_plan_autotune: times the candidate launch layouts on this very batch and keeps
        # the fastest (every layout computes identical bits); part of warmup, not timed.
        progress("autotune")
        plan.autotune(pose_in.data_ptr(), targets.data_ptr(), pose_out.data_ptr(), 0, n, stream.cuda_stream)
        info = plan.info()
    progress(f"warmup {args.warmup}, timed {args.steps}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    elapsed = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    wall_max = float(elapsed.item())

    gather = None
    if dist:
        gather = timed_gathers(pose_out, total, dist, lambda: torch.cuda.synchronize(dev), torch.device(dev))

    # PCIe-inclusive rate (host buffers in, solve, host buffers out): reported, never `value`
    pcie = None
    if rank == 0 and args.pmc != "child":
        plan.solve_host(wl.pose, wl.targets)
        reps = 5
        h0 = time.perf_counter()
        for _ in range(reps):
            plan.solve_host(wl.pose, wl.targets)
        hms = (time.perf_counter() - h0) / reps * 1e3
        pcie = {"ms_per_frame": hms, "skeletons_per_s": n / (hms * 1e-3),
                "note": "mbik_solve_host: pageable host pose/targets in, solve, poses out"}

    # parity spot check against the oracle (not timed): this rank's first 32 and last 32
    # skeletons, so the largest per-skeleton offsets of the timed launch are checked too
    parity = None
    if not args.no_parity and rank == 0 and args.pmc != "child":
        progress("parity")
        try:
            from oracle import pyoracle as po
            head = min(32, n)
            tail = min(32, n - head)
            windows = [(0, head)] + ([(n - tail, tail)] if tail else [])
            gots, refs = [], []
            for lo, k in windows:
                sub = W.generate(cfg, k, first=first + lo)
                o = po.Oracle(sub, **flags)
                refs.append(o.solve(sub.pose, sub.targets, threads=16))
                o.close()
                if args.constraint_mode:  # frames advance the node caches: compare a fresh first frame
                    sp = Plan.from_workload(sub, device=local_rank, **flags)
                    gots.append(sp.solve_host(sub.pose, sub.targets))
                    sp.close()
                else:
                    gots.append(pose_out[lo:lo + k].cpu().numpy())
            got, ref = np.concatenate(gots), np.concatenate(refs)
            qe = quat_error(got, ref)
            parity = {"skeletons": int(got.shape[0]), "ranges": [[first + lo, first + lo + k] for lo, k in windows],
                      "max_quat_err": float(qe.max()),
                      "frac_skeletons_le_1e-4": float(np.mean(qe.max(-1) <= 1e-4)),
                      "bitwise_equal": bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))}
        except Exception as e:  # oracle missing on the box: report, never fall back
            parity = {"error": str(e)}

    # the library's single-process multi-GPU path (mbik_multi_*), after everything above
    lib_multi = None
    lm_devices = [int(x) for x in args.library_multi_devices.split(",") if x] or (list(range(world)) if world > 1 else [])
    if lm_devices and not args.constraint_mode:
        if dist:
            dist.barrier(group=host_group)
        if rank == 0:
            try:
                progress("library_multi")
                lib_multi = library_multi(cfg, [total // len(lm_devices)] * len(lm_devices), lm_devices, args, info, flags)
            except Exception as e:  # noqa: BLE001 -- measurement only: reported, never part of `value`
                lib_multi = {"error": f"{type(e).__name__}: {e}"}
        if dist:
            dist.barrier(group=host_group)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    ms_per_step = wall_max / args.steps * 1e3
    value = total / (wall_max / args.steps)
    alg_bytes = info["algorithmic_bytes_per_skeleton"] * n
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    alg_flops = info["algorithmic_flops_per_skeleton"] * n
    traffic = None
    # committed PMC evidence is keyed by config, size and kernel variant (the plain solve has
    # no suffix): a constraint_mode or stabilization run never borrows the plain kernel's
    key = f"c{cfg}_{n}" + ("_cmode" if args.constraint_mode else "") + \
        (f"_stab{args.stabilization_passes}" if args.stabilization_passes else "")
    # the PMC traffic of exactly the layout timed here (autotune may pick differently per box)
    tkey = key + "_" + layout_key(info)
    live = None
    if pmc_enabled(args, world):
        progress("live counter passes")
        live = live_pmc(args, info, cfg, n)
    traffic_source = None
    if live and "hbm_bytes_per_launch" in live:
        traffic, traffic_source = live["hbm_bytes_per_launch"], "pmc (this run: rocprofv3 --pmc children, pmc_live)"
    elif os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tkey in tj:
                traffic, traffic_source = tj[tkey]["hbm_bytes_per_launch"], "profiles/traffic.json (committed, same layout key)"
        except Exception:
            traffic = None
    issue = None  # the single-wave VALU issue ceiling, from the committed PMC passes
    if os.path.exists(args.valu_mix_json):
        try:
            vm = json.load(open(args.valu_mix_json)).get(tkey)  # the mix of exactly this layout
            if vm and "solver_issue_frac" in vm:
                # helper-wave layout: the solving wave's own instructions (replay launch) over its
                # cycles; the helper's share beside it (tools/replay_count.sh, tools/solver_issue.py)
                issue = {"bound": "valu_issue_1wave", "wave": "solving",
                         "achieved_cycles_per_wave": vm["solver_valu_issue_floor_cycles"],
                         "valu_insts_per_wave": vm["solver_valu_insts_per_wave"],
                         "wave_cycles": vm["solver_wave_cycles"], "frac": vm["solver_issue_frac"],
                         "helper_valu_insts_per_wave": vm["helper_valu_insts_per_wave"],
                         "helper_frac": vm["helper_issue_frac"],
                         "note": "4 cycles per wave64 VALU instruction x the SOLVING wave's VALU instructions (counted on "
                                 "a replay launch of that wave alone, bitwise-equal output) / its wave cycles in the "
                                 "helper-wave launch (PMC, profiles/valu_mix.json); the ceiling this latency-bound "
                                 "chain runs against"}
            elif vm:
                issue = {"bound": "valu_issue_1wave", "achieved_cycles_per_wave": vm["valu_issue_floor_cycles"],
                         "wave_cycles": vm["wave_cycles"], "frac": vm["issue_frac"],
                         "note": "4 cycles per wave64 VALU instruction x VALU instructions / wave cycles (PMC, "
                                 "profiles/valu_mix.json); the ceiling this latency-bound chain runs against"
                                 + ("; helper-wave layout: the mean of the solving wave and its helper"
                                    if info.get("helper_wave") else "")}
        except Exception:
            issue = None
    if issue is not None:
        issue["source"] = "profiles/valu_mix.json (committed, same layout key)"
    pw = (live or {}).get("per_wave") if live and "hbm_bytes_per_launch" in live else None
    if pw and pw.get("issue_frac") and not info.get("helper_wave"):
        # one kind of wave per block: this run's own counters replace the committed mix
        issue = {"bound": "valu_issue_1wave", "achieved_cycles_per_wave": 4 * pw["valu_insts"],
                 "valu_insts_per_wave": pw["valu_insts"], "wave_cycles": pw["wave_cycles"], "frac": pw["issue_frac"],
                 "source": "pmc_live (this run)",
                 "note": "4 cycles per wave64 VALU instruction x VALU instructions / wave cycles; the ceiling this "
                         "latency-bound chain runs against"}
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "skeletons/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded generator, many_bone_ik_amd/workloads.py)",
        "config": {"workload": W.bench_config_name(cfg) + (" + constraint_mode" if args.constraint_mode else "") +
                               (f" + stabilization_passes={args.stabilization_passes}" if args.stabilization_passes else ""),
                   "baseline_config": f"configs[{cfg - 1}]",
                   "skeletons_total": total, "skeletons_per_gpu": n, "bones": wl.bone_count, "effectors": int(wl.topo.pins.shape[0]),
                   "cones_per_bone": wl.topo.cones_per_bone, "iterations": wl.topo.iterations,
                   # bone-steps per iteration on the longest root->leaf path (the latency chain);
                   # SURVEY §8 sized its spine topology at the second figure (why
                   # the rig hangs its chains off one root bone instead)
                   "critical_path_steps": W.critical_path_steps(wl.topo),
                   "survey_critical_path_steps": W.SURVEY_CRITICAL_PATH[cfg],
                   "lanes_per_skeleton": info["lanes_per_skeleton"], "skeletons_per_block": info["skeletons_per_block"],
                   "lds_bytes_per_block": info["lds_bytes_per_block"],
                   "layout": {k: info[k] for k in ("checkpoint_interval", "heading_staging", "state_placement",
                                                   "waves_per_simd", "helper_wave", "wave_roles")},
                   "parallelism": f"dp{world} (skeleton shards, no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_key": tkey, "traffic_source": traffic_source,
                     "algorithmic_bytes_per_launch": alg_bytes, "kernel_ms": kernel_ms,
                     "note": "latency/VALU-bound serial chain; HBM fraction reported as requested (DESIGN.md §5)"},
        "valu": {"achieved": alg_flops / (kernel_ms * 1e-3) / 1e12, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": alg_flops / (kernel_ms * 1e-3) / 1e12 / VALU_PEAK_TFLOPS,
                 "algorithmic_flops_per_launch": alg_flops,
                 "note": "SURVEY.md §8(d) flop formula; the bound that applies to this path (DESIGN.md §5)"},
        "issue": issue,
        "gather_ms": gather["all_gather"]["ms"] if gather else None,
        "gather_to_root_ms": gather["to_root"].get("ms", gather["to_root"].get("error")) if gather else None,
        "gather": gather,
        "pcie_inclusive": pcie,
        "parity": parity,
    }
    if live is not None:
        out["pmc_live"] = live
    if lib_multi is not None:
        out["library_multi"] = lib_multi
    if world > 1:
        out["backend"] = backend
    if os.environ.get("MBIK_BENCH_DEVICE"):
        out["rehearsal"] = f"all {world} ranks on cuda:{local_rank} (MBIK_BENCH_DEVICE): not a scaling measurement"
    if world == 1 and not args.no_cpu_baseline:
        try:
            progress("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds, **flags)
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)}
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def pin_layout(plan, info: dict) -> None:
    """Pins a plan to the launch layout another plan's mbik_plan_info reports."""
    plan.set_helper_wave(info["helper_wave"])
    plan.set_wave_roles(info["wave_roles"])
    plan.set_layout(info["lanes_per_skeleton"], info["skeletons_per_block"], info["checkpoint_interval"])
    plan.set_heading_staging(info["heading_staging"])
    plan.set_locals_placement(info["state_placement"])
    plan.set_waves_per_simd(info["waves_per_simd"])


def library_multi(cfg: int, counts, devices, args, info: dict, flags: dict) -> dict:
    """SURVEY §8(e) through the library alone, as a single-process engine (Godot) would drive it:
    one plan per device in `devices` (plan i owns skeletons [sum(counts[:i]), +counts[i]) of one
    batch), mbik_multi_solve with the whole batch's inputs and outputs on device 0 -- the shards
    go to their devices by peer copies, solve, and the poses come back by peer copies (no
    collective).  Each plan runs the layout the timed rank-0 plan chose.  Times `args.steps`
    frames after `args.warmup`, on device 0's stream (wall clock with a synchronize on both
    sides, and HIP events), and checks the gathered poses' first and last skeletons against the
    oracle."""
    import torch
    from many_bone_ik_amd import workloads as W
    from many_bone_ik_amd.solver import Multi, Plan, quat_error
    total = int(sum(counts))
    t_gen = time.perf_counter()
    wl = W.generate(cfg, total)
    gen_s = time.perf_counter() - t_gen
    plans, lo = [], 0
    for d, c in zip(devices, counts):
        p = Plan(wl.topo.parents, wl.pins(), wl.constraints(), wl.pose[lo:lo + c], wl.cones[lo:lo + c], wl.twist[lo:lo + c],
                 iterations=wl.topo.iterations, default_damp=wl.default_damp, max_cones=wl.cones.shape[2], device=d, **flags)
        pin_layout(p, info)
        plans.append(p)
        lo += c
    m = Multi(plans, root_device=0)
    root = torch.device("cuda", 0)
    pi = torch.from_numpy(wl.pose).to(root)
    tg = torch.from_numpy(wl.targets).to(root)
    po = torch.empty_like(pi)
    st = torch.cuda.Stream(root)
    for _ in range(max(1, args.warmup)):
        m.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), st.cuda_stream)
    for d in sorted(set(devices)):
        torch.cuda.synchronize(torch.device("cuda", d))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(args.steps):
        m.solve(pi.data_ptr(), tg.data_ptr(), po.data_ptr(), st.cuda_stream)
    e1.record(st)
    st.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    ev_ms = e0.elapsed_time(e1) / args.steps
    out = {"devices": devices, "skeletons": total, "plans": len(plans), "steps": args.steps,
           "ms_per_frame": wall * 1e3, "event_ms_per_frame": ev_ms, "skeletons_per_s": total / wall,
           "layout": {k: info[k] for k in ("lanes_per_skeleton", "skeletons_per_block", "checkpoint_interval", "heading_staging",
                                           "state_placement", "waves_per_simd", "helper_wave", "wave_roles")},
           "generate_s": gen_s,
           "note": "mbik_multi_solve (one process, plan per device, peer-copy scatter/gather to device 0); "
                   "a separate measurement, never `value`"}
    if not args.no_parity:
        from oracle import pyoracle as po_
        got_all = po.cpu().numpy()
        checks = []
        for a, k in ((0, min(16, total)), (max(0, total - 16), min(16, total))):
            sub = W.generate(cfg, k, first=a)
            o = po_.Oracle(sub, **flags)
            ref = o.solve(sub.pose, sub.targets, threads=16)
            o.close()
            got = got_all[a:a + k]
            checks.append({"range": [a, a + k], "max_quat_err": float(quat_error(got, ref).max()),
                           "bitwise_equal": bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))})
        out["parity"] = checks
    m.close()
    for p in plans:
        p.close()
    return out


def layout_key(info: dict) -> str:
    """The launch layout a plan runs (mbik_plan_info), as the suffix of profiles/traffic.json keys."""
    return (f"K{info['lanes_per_skeleton']}_s{info['skeletons_per_block']}_i{info['checkpoint_interval']}"
            f"_st{info['heading_staging']}_pl{info['state_placement']}_w{info['waves_per_simd']}"
            + ("_h1" if info.get("helper_wave") else "") + ("_rw" if info.get("wave_roles") else ""))


LAYOUT_FIELDS = ("lanes_per_skeleton", "skeletons_per_block", "checkpoint_interval", "heading_staging", "state_placement",
                 "waves_per_simd", "helper_wave", "wave_roles")
# one rocprofv3 --pmc pass each (FETCH_SIZE takes 3 of the 4 TCC counters, WRITE_SIZE 2)
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",), ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VALU"))


def pmc_enabled(args, world: int) -> bool:
    """The live counter leg runs at N = 1 only, never inside a run that is itself profiled."""
    import shutil
    if args.pmc in ("off", "child") or world > 1:
        return False
    if args.pmc == "on":
        return True
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return False
    return shutil.which("rocprofv3") is not None


def live_pmc(args, info: dict, cfg: int, n: int) -> dict:
    """roofline.traffic and the VALU issue of THIS run's timed layout, measured rather than looked
    up: after the timed region, rank 0 re-runs the same batch on the same layout in child
    processes under `rocprofv3 --pmc` (one pass per counter group, each under its own KILL
    time limit), and averages the solve kernel's timed dispatches.  HBM bytes per launch =
    FETCH_SIZE x 2 + WRITE_SIZE (KB, gfx950 correction of MI355X_MICROARCH.md's HBM section;
    calibrated for this kernel's loads in profiles/r03_fetch_calib.json).  constraint_mode
    children autotune on their own (its frame-dependent layouts are not pinned by --layout); their
    counters are used only when they land on the parent's layout."""
    import shutil
    import tempfile
    layout = ":".join(str(int(info[k])) for k in LAYOUT_FIELDS)
    child = [sys.executable, os.path.abspath(__file__), "--config", str(cfg), "--skeletons", str(n), "--steps", "3",
             "--warmup", "1", "--no-cpu-baseline", "--no-parity", "--pmc", "child"]
    child += ["--constraint-mode"] if args.constraint_mode else ["--layout", layout]
    if args.stabilization_passes:
        child += ["--stabilization-passes", str(args.stabilization_passes)]
    kern = "mbik_cmode_kernel" if args.constraint_mode else "mbik_solve_kernel"
    tmp = tempfile.mkdtemp(prefix="mbik_pmc_", dir="/tmp")
    try:
        return _live_pmc_passes(child, kern, tmp, info)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def counter_means(paths, kern: str, ctrs, last: int = 3):
    """Per counter, the mean over the last `last` dispatches of kernels whose name contains
    `kern` in rocprofv3 counter_collection CSVs (a dispatch's rows are summed: one per counter
    instance); None if no such dispatch."""
    import csv
    per = {}
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                if kern in row["Kernel_Name"]:
                    c = per.setdefault(int(row["Dispatch_Id"]), {})
                    c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    timed = [per[k] for k in sorted(per)[-last:]]
    if not timed:
        return None
    return {ctr: sum(t.get(ctr, 0.0) for t in timed) / len(timed) for ctr in ctrs}


def _live_pmc_passes(child, kern: str, tmp: str, info: dict) -> dict:
    import glob
    import subprocess
    env = dict(os.environ, TMPDIR="/tmp")
    sums, keys = {}, set()
    t0 = time.perf_counter()
    for i, ctrs in enumerate(PMC_PASSES):
        d = os.path.join(tmp, f"p{i}")
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", *ctrs, "-d", d, "-o", "run", "--output-format", "csv",
               "--", *child]
        r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True)
        if r.returncode != 0:
            return {"error": f"pass {' '.join(ctrs)}: exit {r.returncode}: {r.stderr.strip()[-300:]}"}
        try:
            keys.add(json.loads(r.stdout.strip().splitlines()[-1])["roofline"]["traffic_key"])
        except Exception:  # noqa: BLE001
            return {"error": f"pass {' '.join(ctrs)}: no bench line from the child"}
        mean = counter_means(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True), kern, ctrs)
        if mean is None:
            return {"error": f"pass {' '.join(ctrs)}: no {kern} dispatches in the counter CSV"}
        sums.update(mean)
    out = {"passes": [" ".join(c) for c in PMC_PASSES], "dispatches_averaged": 3, "child_layout_keys": sorted(keys),
           "seconds": round(time.perf_counter() - t0, 1), "fetch_size_kb": sums["FETCH_SIZE"], "write_size_kb": sums["WRITE_SIZE"]}
    tkey_parent = layout_key(info)
    if not all(k.endswith(tkey_parent) for k in keys):
        out["error"] = f"child layouts {sorted(keys)} differ from the timed layout {tkey_parent}"
        return out
    out["hbm_bytes_per_launch"] = sums["FETCH_SIZE"] * 1024 * 2 + sums["WRITE_SIZE"] * 1024
    out["correction"] = "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KB x 1024"
    w = max(sums["SQ_WAVES"], 1.0)
    cyc = sums["SQ_WAVE_CYCLES"] * 4 / w  # SQ_WAVE_CYCLES counts 4-cycle units
    valu = sums["SQ_INSTS_VALU"] / w
    out["per_wave"] = {"waves": sums["SQ_WAVES"], "wave_cycles": cyc, "valu_insts": valu,
                       "issue_frac": 4 * valu / cyc if cyc else None,
                       "wait_any_frac": sums["SQ_WAIT_ANY"] / sums["SQ_WAVE_CYCLES"] if sums["SQ_WAVE_CYCLES"] else None,
                       "note": "4 cycles per wave64 VALU instruction x VALU instructions / wave cycles; helper-wave "
                               "layouts: the mean over the solving wave and its helper (the solving wave alone: `issue`)"}
    return out


def timed_gathers(pose_out, total: int, dist, sync, dev) -> dict:
    """Times SURVEY §8(e)'s final gather of the output poses two ways, after the solve loop and
    outside `value`, and reports what each moves: `all_gather` (RCCL all_gather: every rank gets
    every pose) and `to_root` (dist.gather: each peer sends its shard to rank 0 over its own
    xGMI link).  Shards are padded to the largest for one fixed-size collective, so the bytes
    below are the padded messages.  ms = max over ranks; GB/s = bytes received by the busiest
    receiver / ms."""
    import torch
    from many_bone_ik_amd.dist import gather_poses, gather_poses_to_root, shard_range
    world = dist.get_world_size()
    per_skel = int(pose_out[0].numel() * pose_out.element_size()) if pose_out.shape[0] else 0
    cmax = max(shard_range(r, world, total)[1] for r in range(world))
    msg = cmax * per_skel                 # one rank's (padded) shard
    recv = (world - 1) * msg              # what the busiest receiver takes in

    def timed(fn):
        dist.barrier()
        sync()
        g0 = time.perf_counter()
        fn()
        sync()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        return float(gt.item()) * 1e3

    out = {"pose_bytes_total": total * per_skel, "shard_bytes_padded": msg}
    ms = timed(lambda: gather_poses(pose_out, total))
    out["all_gather"] = {"ms": ms, "bytes_in_per_rank": recv, "bytes_out_per_rank": msg,
                         "GBps_in_per_rank": recv / (ms * 1e-3) / 1e9 if ms > 0 else None}
    try:
        ms = timed(lambda: gather_poses_to_root(pose_out, total, root=0))
        out["to_root"] = {"ms": ms, "bytes_in_root": recv, "bytes_out_per_peer": msg,
                          "GBps_in_root": recv / (ms * 1e-3) / 1e9 if ms > 0 else None}
    except Exception as e:  # noqa: BLE001 -- measurement only: reported, never part of `value`
        out["to_root"] = {"error": str(e)}
    return out


def batch_shard(args, world: int, rank: int):
    """(total skeletons, this rank's first, this rank's count) for --scaling."""
    from many_bone_ik_amd.dist import shard_range
    if args.scaling == "weak":
        per = args.skeletons or SKEL_PER_GPU[args.config]
        return per * world, rank * per, per
    total = args.skeletons or SKEL_TOTAL[args.config]
    first, count = shard_range(rank, world, total)
    return total, first, count


def dry_run(args, world: int, rank: int):
    """The multi-rank plumbing without a GPU: gloo rendezvous, this rank's shard, barrier +
    max-over-ranks timing of no-op steps, the pose gather, and rank 0's JSON line."""
    import torch
    import torch.distributed as dist
    from many_bone_ik_amd.dist import gather_poses
    if world > 1:
        dist.init_process_group("gloo")
    total, first, n = batch_shard(args, world, rank)
    shard = torch.arange(first, first + n, dtype=torch.float32).reshape(n, 1, 1).expand(n, 1, 10).contiguous()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    full = gather_poses(shard, total) if world > 1 else shard
    ok = bool(torch.equal(full[:, 0, 0], torch.arange(total, dtype=torch.float32)))
    gather = timed_gathers(shard, total, dist, lambda: None, torch.device("cpu")) if world > 1 else None
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "skeletons/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "scaling": args.scaling, "dry_run": True,
                          "config": {"skeletons_total": total, "skeletons_per_gpu": n},
                          "gathered_in_order": ok, "max_wall_s": float(el.item()), "gather": gather}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
