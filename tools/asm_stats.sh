#!/bin/bash
# Device assembly of solve.hip plus per-kernel register / scratch usage: tools/asm_stats.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
mkdir -p build/asm
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -Wno-unused-result --cuda-device-only -S \
  "$@" many_bone_ik_amd/csrc/solve.hip -o build/asm/solve.s 2>/dev/null
python3 - <<'PY'
import re
txt = open("build/asm/solve.s").read()
meta = txt[txt.index("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    n = f.get("name", "?")
    if any(k in n for k in ("solve_kernel", "group_kernel", "cmode_kernel")):
        print(n.replace("_ZN12_GLOBAL__N_1", "")[:40], {k: f.get(k) for k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count")})
PY
