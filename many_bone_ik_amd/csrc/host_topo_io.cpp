// Plans built on the GPU (topo.h + mbik_setup_kernel: a crowd of distinct rigs in one launch,
// DESIGN.md §10 f1) and plan serialisation (mbik_plan_save / mbik_plan_load).
#include "host.h"

using namespace mbik_host;

// ---- GPU-side topology build (topo.h) ----
namespace {
// Builds the topologies of n rigs with topo.h -- on `device`, one GPU thread per rig, or on
// the host when device < 0 (the same code; the CPU tests use it) -- and assembles each into
// a HostPlan's topology.  errs[i] is the rig's error, empty when it built.
int build_topologies(int n, const mbik_skeleton_desc *descs, const mbik_config *cfgs, int device,
		std::vector<mbik::HostPlan> &out, std::vector<std::string> &errs) {
	out.assign(n, mbik::HostPlan{});
	errs.assign(n, std::string());
	std::vector<mbik::TopoSizes> sz(n);
	std::vector<size_t> in_i(n + 1, 0), in_f(n + 1, 0), in_d(n + 1, 0), o_i(n + 1, 0), o_d(n + 1, 0), o_f(n + 1, 0),
			s_i(n + 1, 0), s_d(n + 1, 0);
	std::vector<char> ok(n, 0);
	for (int i = 0; i < n; i++) {
		const mbik_skeleton_desc &d = descs[i];
		const mbik_config &c = cfgs[i];
		// build_topology's argument checks, in its order (the device never reads a bad pointer)
		if (d.bone_count <= 0 || !d.parents) errs[i] = "bone_count must be > 0 and parents non-null";
		else if (d.pin_count < 0 || (d.pin_count > 0 && !d.pins)) errs[i] = "invalid pins";
		else if (d.constraint_count < 0 || (d.constraint_count > 0 && !d.constraints)) errs[i] = "invalid constraints";
		else if (c.iterations_per_frame < 0) errs[i] = "iterations_per_frame must be >= 0";
		else if (c.bone_damp_count < 0) errs[i] = "negative count"; // (keep_inputs would read a reversed range)
		ok[i] = errs[i].empty();
		const int B = ok[i] ? d.bone_count : 1, P = ok[i] ? d.pin_count : 0, C = ok[i] ? d.constraint_count : 0;
		sz[i] = mbik::topo_sizes(B, P, C);
		in_i[i + 1] = in_i[i] + mbik::topo_align4((size_t)B + P + 2 * (size_t)C);
		in_f[i + 1] = in_f[i] + mbik::topo_align4(5 * (size_t)P);
		in_d[i + 1] = in_d[i] + mbik::topo_align4((size_t)B);
		o_i[i + 1] = o_i[i] + sz[i].out_ints;
		o_d[i + 1] = o_d[i] + sz[i].out_dbls;
		o_f[i + 1] = o_f[i] + sz[i].out_flts;
		s_i[i + 1] = s_i[i] + sz[i].scr_ints;
		s_d[i + 1] = s_d[i] + sz[i].scr_dbls;
	}
	std::vector<int32_t> hin_i(in_i[n] + 4), hout_i(o_i[n] + 4);
	std::vector<float> hin_f(in_f[n] + 4), hout_f(o_f[n] + 4);
	std::vector<double> hin_d(in_d[n] + 4), hout_d(o_d[n] + 4);
	std::vector<double> root_chd(n, 0.0);
	for (int i = 0; i < n; i++) {
		if (!ok[i]) continue;
		const mbik_skeleton_desc &d = descs[i];
		const int B = d.bone_count, P = d.pin_count, C = d.constraint_count;
		int32_t *ii = hin_i.data() + in_i[i];
		float *ff = hin_f.data() + in_f[i];
		std::copy(d.parents, d.parents + B, ii);
		for (int e = 0; e < P; e++) {
			ii[B + e] = d.pins[e].bone;
			ff[e] = d.pins[e].weight;
			for (int a = 0; a < 3; a++) ff[P + 3 * e + a] = d.pins[e].direction_priorities[a];
			ff[4 * P + e] = d.pins[e].motion_propagation_factor;
		}
		for (int c = 0; c < C; c++) {
			ii[B + P + c] = d.constraints[c].bone;
			ii[B + P + C + c] = d.constraints[c].cone_count;
		}
		std::vector<double> chd;
		mbik::topology_damp_cosines(d, cfgs[i], chd, root_chd[i]);
		std::copy(chd.begin(), chd.begin() + B, hin_d.data() + in_d[i]);
	}
	// the slices, pointing into device buffers (or into host buffers when device < 0)
	char *dbase = nullptr;
	std::vector<int32_t> hscr_i;
	std::vector<double> hscr_d;
	const size_t b_in_i = hin_i.size() * 4, b_in_f = hin_f.size() * 4, b_in_d = hin_d.size() * 8, b_o_i = hout_i.size() * 4,
				 b_o_f = hout_f.size() * 4, b_o_d = hout_d.size() * 8, b_s_i = (s_i[n] + 4) * 4, b_s_d = (s_d[n] + 4) * 8,
				 b_sl = (size_t)n * sizeof(TopoSlice);
	auto a16 = [](size_t x) { return (x + 255) & ~size_t(255); };
	const size_t off_in_f = a16(b_in_i), off_in_d = off_in_f + a16(b_in_f), off_o_i = off_in_d + a16(b_in_d),
				 off_o_f = off_o_i + a16(b_o_i), off_o_d = off_o_f + a16(b_o_f), off_s_i = off_o_d + a16(b_o_d),
				 off_s_d = off_s_i + a16(b_s_i), off_sl = off_s_d + a16(b_s_d), total = off_sl + a16(b_sl);
	const bool on_device = device >= 0;
	if (on_device) {
		if (hipMalloc(&dbase, total) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc topology build");
	} else {
		hscr_i.assign(s_i[n] + 4, 0);
		hscr_d.assign(s_d[n] + 4, 0.0);
	}
	auto P_i = [&](size_t off, std::vector<int32_t> &h) { return on_device ? reinterpret_cast<int32_t *>(dbase + off) : h.data(); };
	auto P_f = [&](size_t off, std::vector<float> &h) { return on_device ? reinterpret_cast<float *>(dbase + off) : h.data(); };
	auto P_d = [&](size_t off, std::vector<double> &h) { return on_device ? reinterpret_cast<double *>(dbase + off) : h.data(); };
	int32_t *bin_i = P_i(0, hin_i), *bout_i = P_i(off_o_i, hout_i), *bscr_i = P_i(off_s_i, hscr_i);
	float *bin_f = P_f(off_in_f, hin_f), *bout_f = P_f(off_o_f, hout_f);
	double *bin_d = P_d(off_in_d, hin_d), *bout_d = P_d(off_o_d, hout_d), *bscr_d = P_d(off_s_d, hscr_d);
	std::vector<TopoSlice> slices(n);
	for (int i = 0; i < n; i++) {
		const mbik_skeleton_desc &d = descs[i];
		const int B = ok[i] ? d.bone_count : 0, P = ok[i] ? d.pin_count : 0, C = ok[i] ? d.constraint_count : 0;
		mbik::TopoRig &r = slices[i].rig;
		r.B = B;
		r.P = P;
		r.C = C;
		r.max_cones = d.max_cones;
		r.stab = cfgs[i].stabilization_passes;
		r.parents = bin_i + in_i[i];
		r.pin_bone = bin_i + in_i[i] + B;
		r.cons_bone = bin_i + in_i[i] + B + P;
		r.cons_ncones = bin_i + in_i[i] + B + P + C;
		r.pin_weight = bin_f + in_f[i];
		r.pin_prio = bin_f + in_f[i] + P;
		r.pin_mpf = bin_f + in_f[i] + 4 * P;
		r.bone_chd = bin_d + in_d[i];
		r.root_chd = root_chd[i];
		slices[i].out_i = bout_i + o_i[i];
		slices[i].out_d = bout_d + o_d[i];
		slices[i].out_f = bout_f + o_f[i];
		slices[i].scr_i = bscr_i + s_i[i];
		slices[i].scr_d = bscr_d + s_d[i];
	}
	if (on_device) {
		DeviceGuard guard(device);
		int rc = MBIK_OK;
		if (hipMemcpy(dbase, hin_i.data(), b_in_i, hipMemcpyHostToDevice) != hipSuccess ||
				hipMemcpy(dbase + off_in_f, hin_f.data(), b_in_f, hipMemcpyHostToDevice) != hipSuccess ||
				hipMemcpy(dbase + off_in_d, hin_d.data(), b_in_d, hipMemcpyHostToDevice) != hipSuccess ||
				hipMemcpy(dbase + off_sl, slices.data(), b_sl, hipMemcpyHostToDevice) != hipSuccess)
			rc = fail(MBIK_EHIP, "hipMemcpy topology inputs");
		if (rc == MBIK_OK) {
			if (mbik::launch_topology(reinterpret_cast<const TopoSlice *>(dbase + off_sl), n) != hipSuccess ||
					hipDeviceSynchronize() != hipSuccess)
				rc = fail(MBIK_EHIP, "topology kernel");
		}
		if (rc == MBIK_OK && (hipMemcpy(hout_i.data(), dbase + off_o_i, b_o_i, hipMemcpyDeviceToHost) != hipSuccess ||
								 hipMemcpy(hout_f.data(), dbase + off_o_f, b_o_f, hipMemcpyDeviceToHost) != hipSuccess ||
								 hipMemcpy(hout_d.data(), dbase + off_o_d, b_o_d, hipMemcpyDeviceToHost) != hipSuccess))
			rc = fail(MBIK_EHIP, "hipMemcpy topology outputs");
		(void)hipFree(dbase);
		if (rc) return rc;
	} else {
		for (int i = 0; i < n; i++) {
			const mbik::TopoRig &r = slices[i].rig;
			if (!ok[i]) continue;
			mbik::topo_build(r, mbik::topo_out_at(slices[i].out_i, slices[i].out_d, slices[i].out_f, r.B, r.P, r.C),
					mbik::topo_scratch_at(slices[i].scr_i, slices[i].scr_d, r.B, r.P));
		}
	}
	for (int i = 0; i < n; i++) {
		if (!ok[i]) continue;
		const mbik_skeleton_desc &d = descs[i];
		const mbik::TopoOut o = mbik::topo_out_at(hout_i.data() + o_i[i], hout_d.data() + o_d[i], hout_f.data() + o_f[i],
				d.bone_count, d.pin_count, d.constraint_count);
		errs[i] = mbik::assemble_topology(o, d, cfgs[i], out[i]);
	}
	return MBIK_OK;
}
} // namespace
extern "C" {

int32_t mbik_selftest_topology(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs, int32_t device,
		int32_t *mismatches) {
	if (n_rigs < 0 || (n_rigs > 0 && (!descs || !configs || !mismatches))) return fail(MBIK_EINVAL, "null argument");
	if (device >= 0) {
		int ndev = 0;
		if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MBIK_ENODEV, "no HIP device visible");
		if (device >= ndev) return fail(MBIK_EINVAL, "device index out of range");
	}
	std::vector<mbik::HostPlan> built;
	std::vector<std::string> errs;
	const int rc = build_topologies(n_rigs, descs, configs, device, built, errs);
	if (rc) return rc;
	std::string report;
	for (int i = 0; i < n_rigs; i++) {
		mbik::HostPlan ref;
		const std::string rerr = mbik::build_topology(descs[i], configs[i], ref);
		if (!rerr.empty() || !errs[i].empty()) {
			// both must refuse the rig, with the same message
			mismatches[i] = rerr == errs[i] ? 0 : 1;
			if (mismatches[i] && report.empty()) report = "rig " + std::to_string(i) + ": '" + rerr + "' vs '" + errs[i] + "'";
			continue;
		}
		std::string first;
		mismatches[i] = mbik::compare_topology(ref, built[i], &first);
		if (mismatches[i] && report.empty()) report = "rig " + std::to_string(i) + ": table " + first;
	}
	g_err = report;
	return MBIK_OK;
}

int32_t mbik_plan_create_device(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs,
		const int32_t *n_skeletons, const float *const *setup_pose, const float *const *cones, const float *const *twist,
		int32_t device, mbik_plan **out_plans) {
	return mbik_plan_create_device_opts(n_rigs, descs, configs, nullptr, n_skeletons, setup_pose, cones, twist, device, out_plans);
}

int32_t mbik_plan_create_device_opts(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs,
		const mbik_plan_options *opts, const int32_t *n_skeletons, const float *const *setup_pose, const float *const *cones,
		const float *const *twist, int32_t device, mbik_plan **out_plans) {
	if (n_rigs <= 0 || !descs || !configs || !n_skeletons || !setup_pose || !out_plans) return fail(MBIK_EINVAL, "null argument");
	for (int i = 0; i < n_rigs; i++) out_plans[i] = nullptr;
	int libm = 0;
	if (read_options(opts, libm)) return MBIK_EINVAL;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MBIK_ENODEV, "no HIP device visible");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device index out of range");
	for (int i = 0; i < n_rigs; i++)
		if (n_skeletons[i] <= 0 || !setup_pose[i]) return fail(MBIK_EINVAL, "n_skeletons must be > 0 and setup_pose non-null");
	std::vector<mbik::HostPlan> built;
	std::vector<std::string> errs;
	int rc = build_topologies(n_rigs, descs, configs, device, built, errs);
	if (rc) return rc;
	for (int i = 0; i < n_rigs; i++)
		if (!errs[i].empty()) return fail(MBIK_EINVAL, "rig " + std::to_string(i) + ": " + errs[i]);
	// every rig's remaining argument checks before any plan takes device memory
	for (int i = 0; i < n_rigs; i++) {
		for (int c : built[i].cons_order_ncones)
			if (c > std::max(1, descs[i].max_cones))
				return fail(MBIK_EINVAL, "rig " + std::to_string(i) + ": a constraint has more cones than max_cones");
		if (built[i].NC > 0 && (!cones || !twist || !cones[i] || !twist[i]))
			return fail(MBIK_EINVAL, "rig " + std::to_string(i) + ": cones/twist required when constraints exist");
	}
	std::vector<std::unique_ptr<mbik_plan>> plans;
	for (int i = 0; i < n_rigs && rc == MBIK_OK; i++) {
		const mbik_skeleton_desc &d = descs[i];
		std::unique_ptr<mbik_plan> p(new mbik_plan());
		p->device = device;
		p->setup_on_device = true;
		keep_inputs(p.get(), d, configs[i]);
		mbik::HostPlan &h = p->host;
		h = std::move(built[i]);
		h.libm_variant = libm;
		h.N = n_skeletons[i];
		const size_t N = (size_t)h.N;
		h.D.assign((size_t)h.B * 9 * N, 0.0f); // filled on the device below (mbik_setup_kernel)
		h.CF.assign((size_t)h.NC * h.cf_stride() * N, 0.0f);
		h.CD.assign((size_t)h.NC * h.cd_stride() * N, 0.0);
		mbik::setup_tables(h);
		h.setup_max_cones = std::max(1, d.max_cones);
		rc = finish_plan(p.get(), setup_pose[i], nullptr); // (frees what it took when it fails)
		if (rc == MBIK_OK)
			rc = mbik_plan_rebuild_setup(p.get(), 0, h.N, setup_pose[i], h.NC ? cones[i] : nullptr, h.NC ? twist[i] : nullptr, nullptr);
		plans.push_back(std::move(p)); // released through mbik_plan_destroy below on any failure
	}
	if (rc) {
		for (auto &p : plans) mbik_plan_destroy(p.release());
		return rc;
	}
	for (int i = 0; i < n_rigs; i++) out_plans[i] = plans[i].release();
	return MBIK_OK;
}

} // extern "C"
// ---- plan serialisation (mbik_plan_save / mbik_plan_load) ----
namespace {
constexpr char kPlanMagic[8] = {'M', 'B', 'I', 'K', 'P', 'L', 'A', 'N'};
constexpr uint32_t kPlanFormat = 5; // 2: + the table-addressing override; 3: + libm_variant, constraint_mode spw; 4: + the helper-wave override; 5: + the wave-roles override (1-4 are still read)
struct PlanWriter {
	std::vector<char> b;
	void bytes(const void *v, size_t n) {
		const char *c = static_cast<const char *>(v);
		b.insert(b.end(), c, c + n);
	}
	template <class T>
	void put(const T &v) { bytes(&v, sizeof(T)); }
	template <class T>
	void vec(const std::vector<T> &v) {
		put<uint64_t>(v.size());
		bytes(v.data(), v.size() * sizeof(T));
	}
};
struct PlanReader {
	const char *p, *e;
	bool ok = true;
	bool bytes(void *v, size_t n) {
		if (!ok || (size_t)(e - p) < n) return ok = false;
		std::memcpy(v, p, n);
		p += n;
		return true;
	}
	template <class T>
	T get() {
		T v{};
		bytes(&v, sizeof(T));
		return v;
	}
	template <class T>
	std::vector<T> vec(uint64_t max_elems) {
		const uint64_t n = get<uint64_t>();
		std::vector<T> v;
		if (!ok || n > max_elems || n > (uint64_t)(e - p) / sizeof(T)) {
			ok = false;
			return v;
		}
		v.resize(n);
		bytes(v.data(), n * sizeof(T));
		return v;
	}
};
size_t cmode_state_bytes(const mbik_plan *p) {
	const mbik::HostPlan &h = p->host;
	return (size_t)(3 * h.B + 2 * h.NC) * 12 * (size_t)h.N * sizeof(float) + 4 * (size_t)p->cm.W * (size_t)h.N * sizeof(uint32_t);
}
} // namespace
extern "C" {

int32_t mbik_plan_save(const mbik_plan *p, void *buf, uint64_t capacity, uint64_t *size) {
	if (!p || !size) return fail(MBIK_EINVAL, "null argument");
	const mbik::HostPlan &h = p->host;
	DeviceGuard guard(p->device);
	// the device tables are read back: every stream that uses the plan must be idle
	if (hipDeviceSynchronize() != hipSuccess) return fail(MBIK_EHIP, "hipDeviceSynchronize");
	PlanWriter w;
	w.bytes(kPlanMagic, sizeof(kPlanMagic));
	w.put<uint32_t>(kPlanFormat);
	w.put<uint32_t>(MBIK_ABI_VERSION);
	w.put<int32_t>(h.N);
	w.vec(p->src_parents);
	w.vec(p->src_pins);
	w.vec(p->src_cons);
	w.put<int32_t>(p->src_max_cones);
	w.put<int32_t>(p->src_cfg.iterations_per_frame);
	w.put<float>(p->src_cfg.default_damp);
	w.put<int32_t>(p->src_cfg.constraint_mode);
	w.put<int32_t>(p->src_cfg.stabilization_passes);
	w.vec(p->src_bone_damp);
	w.put<int32_t>(h.setup_max_cones);
	const size_t N = (size_t)h.N;
	std::vector<float> D((size_t)h.B * 9 * N), CF((size_t)h.NC * h.cf_stride() * N);
	std::vector<double> CD((size_t)h.NC * h.cd_stride() * N);
	if ((!D.empty() && hipMemcpy(D.data(), p->dev.D, D.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) ||
			(!CF.empty() && hipMemcpy(CF.data(), p->dev.CF, CF.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) ||
			(!CD.empty() && hipMemcpy(CD.data(), p->dev.CD, CD.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
		return fail(MBIK_EHIP, "hipMemcpy plan tables");
	w.vec(D);
	w.vec(CF);
	w.vec(CD);
	for (int32_t v : {p->lanes_override, p->spw_override, p->interval_override, p->staging_override, p->locals_override,
				 p->waves_override, p->cm_lanes, p->tab64, p->cm_spw_div})
		w.put<int32_t>(v);
	std::vector<char> cm;
	if (h.constraint_mode && N) {
		cm.resize(cmode_state_bytes(p));
		const size_t node_bytes = cmode_file_node_bytes(h);
		std::vector<float> tiled(node_area_floats(3 * h.B + 2 * h.NC, N));
		if (hipMemcpy(tiled.data(), p->cm.node, tiled.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess ||
				hipMemcpy(cm.data() + node_bytes, p->cm.dirty, cm.size() - node_bytes, hipMemcpyDeviceToHost) != hipSuccess)
			return fail(MBIK_EHIP, "hipMemcpy constraint_mode state");
		cmode_nodes_plain(h, tiled.data(), reinterpret_cast<float *>(cm.data()));
	}
	w.vec(cm);
	w.put<int32_t>(h.libm_variant); // format 3
	w.put<int32_t>(p->helper_override); // format 4
	w.put<int32_t>(p->roles_override); // format 5
	*size = w.b.size();
	if (!buf) return MBIK_OK;
	if (capacity < w.b.size()) return fail(MBIK_EINVAL, "buffer smaller than the saved plan (see *size)");
	std::memcpy(buf, w.b.data(), w.b.size());
	return MBIK_OK;
}

int32_t mbik_plan_load(const void *buf, uint64_t size, int32_t device, mbik_plan **out_plan) {
	if (!buf || !out_plan) return fail(MBIK_EINVAL, "null argument");
	*out_plan = nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MBIK_ENODEV, "no HIP device visible");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device index out of range");
	PlanReader r{static_cast<const char *>(buf), static_cast<const char *>(buf) + size};
	char magic[8];
	if (!r.bytes(magic, 8) || std::memcmp(magic, kPlanMagic, 8) != 0) return fail(MBIK_EINVAL, "not a saved mbik plan");
	const uint32_t format = r.get<uint32_t>();
	if (!r.ok) return fail(MBIK_EINVAL, "truncated or corrupt saved plan");
	if (format < 1 || format > kPlanFormat) return fail(MBIK_EUNSUPPORTED, "saved plan format version not supported");
	(void)r.get<uint32_t>(); // the ABI version that wrote it (informational)
	const int32_t N = r.get<int32_t>();
	constexpr uint64_t kMax = 1ull << 34;
	std::unique_ptr<mbik_plan> p(new mbik_plan());
	p->device = device;
	p->src_parents = r.vec<int32_t>(1 << 24);
	p->src_pins = r.vec<mbik_pin>(1 << 24);
	p->src_cons = r.vec<mbik_constraint>(1 << 24);
	p->src_max_cones = r.get<int32_t>();
	p->src_cfg.iterations_per_frame = r.get<int32_t>();
	p->src_cfg.default_damp = r.get<float>();
	p->src_cfg.constraint_mode = r.get<int32_t>();
	p->src_cfg.stabilization_passes = r.get<int32_t>();
	p->src_bone_damp = r.vec<float>(1 << 24);
	const int32_t setup_max_cones = r.get<int32_t>();
	std::vector<float> D = r.vec<float>(kMax), CF = r.vec<float>(kMax);
	std::vector<double> CD = r.vec<double>(kMax);
	int32_t ov[9] = {};
	for (int i = 0; i < (format >= 3 ? 9 : format == 2 ? 8 : 7); i++) ov[i] = r.get<int32_t>();
	std::vector<char> cm = r.vec<char>(kMax);
	const int32_t libm = format >= 3 ? r.get<int32_t>() : MBIK_LIBM_VARIANT_FMA;
	const int32_t helper = format >= 4 ? r.get<int32_t>() : -1;
	const int32_t roles = format >= 5 ? r.get<int32_t>() : -1;
	if (!r.ok || N <= 0) return fail(MBIK_EINVAL, "truncated or corrupt saved plan");
	if (libm != MBIK_LIBM_VARIANT_FMA && libm != MBIK_LIBM_VARIANT_SSE2) return fail(MBIK_EINVAL, "saved plan: unknown libm_variant");
	if (helper < -1 || helper > 1) return fail(MBIK_EINVAL, "saved plan: unknown helper-wave setting");
	if (roles < -1 || roles > 1) return fail(MBIK_EINVAL, "saved plan: unknown wave-roles setting");
	mbik_skeleton_desc desc{};
	desc.bone_count = (int32_t)p->src_parents.size();
	desc.parents = p->src_parents.data();
	desc.pin_count = (int32_t)p->src_pins.size();
	desc.pins = p->src_pins.data();
	desc.constraint_count = (int32_t)p->src_cons.size();
	desc.constraints = p->src_cons.data();
	desc.max_cones = p->src_max_cones;
	mbik_config cfg = p->src_cfg;
	cfg.bone_damp_count = (int32_t)p->src_bone_damp.size();
	cfg.bone_damp = p->src_bone_damp.empty() ? nullptr : p->src_bone_damp.data();
	p->src_cfg.bone_damp_count = cfg.bone_damp_count;
	mbik::HostPlan &h = p->host;
	std::string err = mbik::build_topology(desc, cfg, h);
	if (!err.empty()) return fail(MBIK_EINVAL, "saved plan: " + err);
	h.libm_variant = libm;
	h.N = N;
	const size_t n = (size_t)N;
	if (D.size() != (size_t)h.B * 9 * n || CF.size() != (size_t)h.NC * h.cf_stride() * n ||
			CD.size() != (size_t)h.NC * h.cd_stride() * n)
		return fail(MBIK_EINVAL, "saved plan tables do not match its topology");
	mbik::setup_tables(h);
	h.setup_max_cones = std::max(1, setup_max_cones);
	h.D = std::move(D);
	h.CF = std::move(CF);
	h.CD = std::move(CD);
	p->lanes_override = ov[0];
	p->spw_override = ov[1];
	p->interval_override = ov[2];
	p->staging_override = ov[3];
	p->locals_override = ov[4];
	p->waves_override = ov[5];
	p->cm_lanes = ov[6];
	p->tab64 = ov[7] != 0;
	p->cm_spw_div = std::max(0, std::min(6, ov[8]));
	p->helper_override = helper;
	p->roles_override = roles;
	if (h.constraint_mode) {
		const int W = std::max(1, (h.cm_npos + 31) / 32);
		const size_t want = (size_t)(3 * h.B + 2 * h.NC) * 12 * n * sizeof(float) + 4 * (size_t)W * n * sizeof(uint32_t);
		if (cm.size() != want) return fail(MBIK_EINVAL, "saved constraint_mode state does not match its topology");
	}
	DeviceGuard guard(device);
	const int rc = finish_plan(p.get(), nullptr, h.constraint_mode ? cm.data() : nullptr);
	if (rc) return rc;
	*out_plan = p.release();
	return MBIK_OK;
}

} // extern "C"
