"""How much does the libm's last ulp move a full solve?  Runs the oracle three ways on the
same inputs and prints the per-config quaternion spread against the default build:
  platform  (default) the platform libm -- glibc 2.35, what a Linux x86-64 Godot build calls;
  restated  -DORACLE_GLIBC_RESTATED: oracle/glibc_libm.h's restatement of glibc's
            sinf/cosf/acosf (expected: bitwise equal to platform);
  pinned    -DORACLE_PINNED_TRIG: round 1's (float)f((double)x) convention.
Usage: python tools/libm_sensitivity.py   (builds the two variant oracles under /tmp first)"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
CASES = [(1, 1), (2, 64), (3, 64), (4, 16), (5, 8)]

if len(sys.argv) > 1 and sys.argv[1] == '--child':
    from many_bone_ik_amd import workloads as W
    from oracle import pyoracle as po
    for cfg, n in CASES:
        wl = W.generate(cfg, n)
        o = po.Oracle(wl)
        np.save(os.path.join(sys.argv[2], f'c{cfg}.npy'), o.solve(wl.pose, wl.targets, threads=8))
    sys.exit(0)


def build(defs, out):
    subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle'), f'ORACLE_DEFS={defs}',
                    f'BUILD={out}'], check=True)
    return os.path.join(out, 'liboracle.so')


from many_bone_ik_amd.solver import quat_error  # noqa: E402

subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle')], check=True)
res = {}
with tempfile.TemporaryDirectory() as tmp:
    libs = {'platform': None,
            'restated': build('-DORACLE_GLIBC_RESTATED', os.path.join(tmp, 'restated')),
            'pinned': build('-DORACLE_PINNED_TRIG', os.path.join(tmp, 'pinned'))}
    outs = {}
    for name, lib in libs.items():
        d = os.path.join(tmp, 'out_' + name)
        os.makedirs(d)
        env = dict(os.environ)
        if lib:
            env['ORACLE_LIB'] = lib
        subprocess.run([sys.executable, __file__, '--child', d], check=True, cwd=ROOT, env=env)
        outs[name] = d
    for name in ('restated', 'pinned'):
        r = {}
        for cfg, n in CASES:
            x = np.load(os.path.join(outs['platform'], f'c{cfg}.npy'))
            y = np.load(os.path.join(outs[name], f'c{cfg}.npy'))
            e = quat_error(x, y)
            r[f'C{cfg}'] = dict(skeletons=n, max_qerr=float(e.max()), frac_skel_le_1e4=float((e.max(1) <= 1e-4).mean()),
                                bitwise_equal=bool(np.array_equal(x.view(np.uint32), y.view(np.uint32))))
        res[f'{name}_vs_platform'] = r
print(json.dumps(res, indent=1))
