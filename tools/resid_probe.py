"""Residency (one-wave blocks per CU) the occupancy query reports for each LDS size of a plan."""
import sys
sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Plan
wl = W.generate(5, 8)
p = Plan.from_workload(wl)
for kb in [40.0, 40.5, 53.0, 53.5, 54.0, 54.6, 79.0, 79.5, 80.0, 80.5, 81.0, 81.5, 82.0]:
    print(kb, p._L.mbik_plan_resident_blocks(p.h, int(kb * 1024)))
