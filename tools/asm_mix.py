"""Static instruction mix of one kernel in build/asm/<tu>.s (run tools/asm_stats.sh first).
    python tools/asm_mix.py [kernel-substring] [build/asm/<tu>.s]"""
import collections
import sys

name = sys.argv[1] if len(sys.argv) > 1 else "mbik_solve_kernelILb0E"
s = open(sys.argv[2] if len(sys.argv) > 2 else "build/asm/k_solve_rw.s").read().split("\n")
start = next(i for i, l in enumerate(s) if name in l and l.split(":")[0].endswith(l.split(":")[0]) and l.startswith("_Z"))
end = next(i for i in range(start, len(s)) if s[i].strip().startswith("s_endpgm") or s[i].startswith(".Lfunc_end"))
c = collections.Counter()
for l in s[start:end]:
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":") or ":" in l.split()[0]:
        continue
    c[l.split()[0]] += 1
tot = sum(c.values())
print("total", tot)
groups = {"accvgpr": lambda o: "accvgpr" in o, "f64": lambda o: "f64" in o, "s_nop": lambda o: o == "s_nop",
          "salu": lambda o: o.startswith("s_"), "ds": lambda o: o.startswith("ds_"),
          "global/buffer": lambda o: o.startswith(("global_", "buffer_", "flat_")),
          "transcendental": lambda o: any(k in o for k in ("rcp", "rsq", "sqrt", "sin", "cos", "log", "exp"))}
for g, f in groups.items():
    print(f"{g:16s}{sum(n for o, n in c.items() if f(o))}")
for o, n in c.most_common(40):
    print(f"  {o:30s}{n}")
