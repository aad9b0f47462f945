"""Static per-loop instruction counts of one kernel in an asm listing (tools/asm_stats.sh output,
or a -gline-tables-only listing for per-source-line attribution).
    python tools/asm_loops.py build/asm/<tu>.s kernel_substring [loop_label_for_line_detail]   (tools/asm_stats.sh -gline-tables-only)"""
import collections
import re
import sys

path, ksub = sys.argv[1], sys.argv[2]
detail = sys.argv[3] if len(sys.argv) > 3 else None
txt = open(path).read()
files = {m.group(1): (m.group(3) or m.group(2)).split('/')[-1]
         for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', txt)}
name = next(m.group(1) for m in re.finditer(r'^(\S*' + re.escape(ksub) + r'\S*):', txt, re.M))
start = txt.index(name + ':')
body = txt[start:txt.index('.Lfunc_end', start)].split('\n')
loops = collections.OrderedDict()
lines = collections.Counter()
cur_loop, cur_src, pending = None, None, None
for ln in body:
    s = ln.strip()
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
    if m:
        cur_src = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    lab = re.match(r'^(?:\.LBB(\d+_\d+):|; %bb\.(\d+):)', s)
    if lab:
        pending = lab.group(1) or ('bb' + lab.group(2))
        cur_loop = None
    if s.startswith(';') or lab:
        h = re.search(r'Loop Header: Depth=(\d+)', s)
        inl = re.search(r'in Loop: Header=BB(\d+_\d+) Depth=(\d+)', s)
        if h and pending:
            cur_loop = (pending, int(h.group(1)))
        elif inl:
            cur_loop = (inl.group(1), int(inl.group(2)))
        continue
    if not s or s.startswith('.'):
        continue
    op = s.split()[0]
    key = cur_loop or ('-', 0)
    c = loops.setdefault(key, collections.Counter())
    c['all'] += 1
    for k in ('v_mov', 'v_pk', 'f64', 'v_readlane', 'v_accvgpr', 's_nop', 's_waitcnt', 'ds_', 'buffer_', 'v_cndmask'):
        if op.startswith(k) or (k == 'f64' and op.endswith('f64')):
            c[k] += 1
    if detail and key[0] == detail:
        lines[cur_src] += 1
for (h, d), c in loops.items():
    print(f"{h:>10} depth {d}: " + " ".join(f"{k}={v}" for k, v in c.items()))
if detail:
    for k, v in lines.most_common(40):
        print(k, v)
