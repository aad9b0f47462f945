// Host plan builder under ASan + UBSan: ManyBoneIK3D::_bone_list_changed's segmentation and
// heading weights (plan.cpp build_topology), the per-skeleton setup on host threads
// (build_skeletons -> setup.h), and every launch schedule the library can pick
// (build_schedule over lane counts, skeletons per block and checkpoint intervals).
//   plan_san <case file>   -> exit 0 and one summary line, or a sanitizer report
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../many_bone_ik_amd/csrc/plan.h"
#include "case_io.h"

int main(int argc, char **argv) {
	if (argc < 2) return 2;
	san_case c = san_load(argv[1]);
	std::vector<mbik_pin> pins(std::max(1, c.P));
	for (int i = 0; i < c.P; i++) {
		pins[i].bone = c.pin_bone[i];
		pins[i].weight = c.pin_weight[i];
		for (int a = 0; a < 3; a++) pins[i].direction_priorities[a] = c.pin_prio[3 * i + a];
		pins[i].motion_propagation_factor = c.pin_prop[i];
	}
	std::vector<mbik_constraint> cons(std::max(1, c.C));
	for (int i = 0; i < c.C; i++) cons[i] = mbik_constraint{c.cons_bone[i], c.cons_ncones[i]};
	mbik_skeleton_desc d{c.B, c.parents, c.P, pins.data(), c.C, cons.data(), c.max_cones};
	mbik_config cfg{c.iterations, c.default_damp, c.constraint_mode, c.stab, c.bone_damp_count,
			c.bone_damp_count ? c.bone_damp : nullptr};
	mbik::HostPlan h;
	std::string err = mbik::build_topology(d, cfg, h);
	if (!err.empty()) {
		printf("build_topology refused: %s\n", err.c_str());
		return 0; // a refused description is a valid outcome; the sanitizers watched the checks
	}
	err = mbik::build_skeletons(h, c.N, c.pose, c.C ? c.cones : nullptr, c.C ? c.twist : nullptr, std::max(1, c.max_cones));
	if (!err.empty()) {
		printf("build_skeletons refused: %s\n", err.c_str());
		return 0;
	}
	int64_t acc = 0;
	for (int lanes : {0, 1, 2, 4, 8, 16, 64})
		for (int interval : {0, 1, 2, 3, 1 << 20})
			for (int spw : {0, 1, 3, 64}) {
				mbik::HostPlan q = h;
				q.state_hbm = (lanes / 2) % 3;
				q.staging = (lanes & 1) == 0 ? 1 : (interval == 2 ? 2 : 0);
				mbik::build_schedule(q, lanes, c.N, spw, interval);
				acc += mbik::lds_floats_per_skeleton(q) + mbik::state_floats_per_skeleton(q) + mbik::topology_bytes(q) + q.nrows;
			}
	double chk = 0;
	for (float v : h.D) chk += v;
	for (float v : h.CF) chk += v;
	for (double v : h.CD) chk += v;
	printf("ok B=%d segments=%d N=%d schedules=%lld checksum=%.6g\n", h.B, h.NS, h.N, (long long)acc, chk);
	san_free(&c);
	return 0;
}
