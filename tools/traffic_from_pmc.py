"""HBM traffic per solve launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB per
dispatch), corrected as /opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes:
FETCH_SIZE x2 on gfx950 (128-B requests tallied at 64 B), WRITE_SIZE as is.  The kernel's
loads are dword-wide, for which the guide calls the x2 uncalibrated; the record says so.

    python tools/traffic_from_pmc.py <fetch_csv> <write_csv> <key> [profiles/traffic.json] [--last N]

--last N averages only the last N solve dispatches (bench.py's timed steps and its host-buffer
frames, after mbik_plan_autotune has fixed the layout; the autotune candidates come first).
"""
import csv, json, os, sys

KERNEL = "mbik_solve_kernel"


def per_dispatch(path, counter, last=0):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                d = int(r["Dispatch_Id"])
                vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {path}")
    keys = sorted(vals)[-last:] if last else sorted(vals)
    return sum(vals[k] for k in keys) / len(keys), len(keys)


def main():
    args = sys.argv[1:]
    last = 0
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    fetch_csv, write_csv, key = args[:3]
    out = args[3] if len(args) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    fk, nf = per_dispatch(fetch_csv, "FETCH_SIZE", last)
    wk, nw = per_dispatch(write_csv, "WRITE_SIZE", last)
    rec = {"fetch_size_kb": fk, "write_size_kb": wk, "dispatches": [nf, nw],
           "read_bytes": fk * 1024 * 2, "write_bytes": wk * 1024,
           "hbm_bytes_per_launch": fk * 1024 * 2 + wk * 1024,
           "correction": "FETCH_SIZE x2 (gfx950, guide HBM section; calibrated for this kernel's b32/b64/b128, tiled and gathered buffer loads in round 3: profiles/r03_fetch_calib.json), KB x1024"}
    tj = json.load(open(out)) if os.path.exists(out) else {}
    tj[key] = rec
    with open(out, "w") as f:
        json.dump(tj, f, indent=1, sort_keys=True)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
