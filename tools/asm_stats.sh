#!/bin/bash
# Device assembly of the solve kernel TUs plus per-kernel register / scratch usage:
#   tools/asm_stats.sh [extra hipcc flags]      -> build/asm/<tu>.s
set -e
cd "$(dirname "$0")/.."
mkdir -p build/asm
for tu in k_solve_w1 k_solve_w2 k_solve_rw k_cmode; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -Wno-unused-result --cuda-device-only -S \
    "$@" many_bone_ik_amd/csrc/$tu.hip -o build/asm/$tu.s 2>/dev/null &
done
wait
python3 - <<'PY'
import re
for tu in ("k_solve_w1", "k_solve_w2", "k_solve_rw", "k_cmode"):
  txt = open(f"build/asm/{tu}.s").read()
  meta = txt[txt.index("amdhsa.kernels:"):]
  for blk in meta.split("\n  - ")[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    n = f.get("name", "?")
    if any(k in n for k in ("solve_kernel", "group_kernel", "cmode_kernel")):
        print(n.replace("_ZN12_GLOBAL__N_1", "")[:40], {k: f.get(k) for k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count")})
PY
