"""How much do 1-ulp differences in sinf/cosf/acosf move a full solve?  Runs the oracle
with transcendentals pinned to (float)f((double)x) (the default, also what the GPU
kernel evaluates) and with the platform's float libm (-DORACLE_PLATFORM_LIBM build named
by ORACLE_LIB), on the same inputs, and prints the per-config quaternion spread.
Usage: python tools/libm_sensitivity.py   (builds oracle/build/liboracle_platlibm.so first)"""
import json, os, subprocess, sys
import numpy as np
sys.path.insert(0, '.')
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PLAT = os.path.join(ROOT, 'oracle', 'build', 'liboracle_platlibm.so')
CASES = [(1, 1), (2, 64), (3, 64), (4, 16), (5, 8)]

if len(sys.argv) > 1 and sys.argv[1] == '--child':
    from many_bone_ik_amd import workloads as W
    from oracle import pyoracle as po
    out = {}
    for cfg, n in CASES:
        wl = W.generate(cfg, n)
        o = po.Oracle(wl)
        np.save(os.path.join(sys.argv[2], f'c{cfg}.npy'), o.solve(wl.pose, wl.targets, threads=8))
    sys.exit(0)

subprocess.run(['gcc', '-O2', '-std=c11', '-fPIC', '-ffp-contract=off', '-fno-fast-math', '-DORACLE_PLATFORM_LIBM',
                '-shared', '-o', PLAT, os.path.join(ROOT, 'oracle', 'ik_oracle.c'), '-lm', '-lpthread'], check=True)
import tempfile
from many_bone_ik_amd.solver import quat_error
res = {}
with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
    subprocess.run([sys.executable, __file__, '--child', a], check=True, cwd=ROOT)
    subprocess.run([sys.executable, __file__, '--child', b], check=True, cwd=ROOT, env=dict(os.environ, ORACLE_LIB=PLAT))
    for cfg, n in CASES:
        x, y = np.load(os.path.join(a, f'c{cfg}.npy')), np.load(os.path.join(b, f'c{cfg}.npy'))
        e = quat_error(x, y)
        res[f'C{cfg}'] = dict(skeletons=n, max_qerr=float(e.max()), frac_skel_le_1e4=float((e.max(1) <= 1e-4).mean()),
                              bitwise_equal=bool((x == y).all()))
print(json.dumps(res, indent=1))
