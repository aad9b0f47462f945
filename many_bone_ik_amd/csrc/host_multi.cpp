// Multi-GPU inside the library (mbik_multi_*): contiguous skeleton shards over
// per-device plans, driven from one host thread, with peer-copy scatter and gather to a root
// device.
#include "host.h"

using namespace mbik_host;

extern "C" {

// ---- Multi-GPU in one process (mbik_multi_*) ----
struct mbik_multi {
	std::vector<mbik_plan *> plans; // not owned
	std::vector<int64_t> off;       // shard offsets, plans.size() + 1
	int root = 0;
	uint32_t flags = 0;
	struct Shard {
		hipStream_t stream = nullptr;
		hipEvent_t done = nullptr;
		bool staged = false;
		float *in = nullptr, *tg = nullptr, *out = nullptr; // staging on the plan's device
	};
	std::vector<Shard> sh;
	hipEvent_t start = nullptr; // on the root device: "the caller's queued work is done"
};

void mbik_multi_destroy(mbik_multi *m) {
	if (!m) return;
	for (size_t i = 0; i < m->sh.size(); i++) {
		auto &s = m->sh[i];
		DeviceGuard g(m->plans[i]->device);
		if (s.stream) (void)hipStreamSynchronize(s.stream);
		if (s.in) (void)hipFree(s.in);
		if (s.tg) (void)hipFree(s.tg);
		if (s.out) (void)hipFree(s.out);
		if (s.done) (void)hipEventDestroy(s.done);
		if (s.stream) (void)hipStreamDestroy(s.stream);
	}
	if (m->start) {
		DeviceGuard g(m->root);
		(void)hipEventDestroy(m->start);
	}
	delete m;
}

int32_t mbik_multi_create(mbik_plan *const *plans, int32_t n_plans, int32_t root_device, uint32_t flags, mbik_multi **out) {
	if (!plans || n_plans <= 0 || !out) return fail(MBIK_EINVAL, "null argument or no plans");
	if (flags & ~MBIK_MULTI_STAGE_ALL) return fail(MBIK_EINVAL, "unknown mbik_multi flags");
	*out = nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MBIK_ENODEV, "no HIP device visible");
	if (root_device < 0 || root_device >= ndev) return fail(MBIK_EINVAL, "root device out of range");
	for (int i = 0; i < n_plans; i++) {
		if (!plans[i]) return fail(MBIK_EINVAL, "null plan");
		for (int j = 0; j < i; j++)
			if (plans[j] == plans[i]) return fail(MBIK_EINVAL, "a plan appears twice");
		if (plans[i]->host.B != plans[0]->host.B || plans[i]->host.P != plans[0]->host.P)
			return fail(MBIK_EINVAL, "multi plans must have the same bone and pin counts");
	}
	std::unique_ptr<mbik_multi, void (*)(mbik_multi *)> m(new mbik_multi(), mbik_multi_destroy);
	m->plans.assign(plans, plans + n_plans);
	m->root = root_device;
	m->flags = flags;
	m->off.assign(1, 0);
	for (mbik_plan *p : m->plans) m->off.push_back(m->off.back() + p->host.N);
	{
		DeviceGuard g(root_device);
		if (hipEventCreateWithFlags(&m->start, hipEventDisableTiming) != hipSuccess) {
			m->start = nullptr;
			return fail(MBIK_EHIP, "hipEventCreate");
		}
	}
	m->sh.resize(n_plans);
	const int B = plans[0]->host.B, P = plans[0]->host.P;
	for (int i = 0; i < n_plans; i++) {
		mbik_plan *p = m->plans[i];
		auto &s = m->sh[i];
		DeviceGuard g(p->device);
		if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) {
			s.stream = nullptr;
			return fail(MBIK_EHIP, "hipStreamCreate");
		}
		if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
			s.done = nullptr;
			return fail(MBIK_EHIP, "hipEventCreate");
		}
		s.staged = p->device != root_device || (flags & MBIK_MULTI_STAGE_ALL);
		if (!s.staged) continue;
		if (p->device != root_device) {
			// peer access both ways where the fabric allows it (xGMI); the peer copies below work
			// without it, through a host-staged path
			int can = 0;
			if (hipDeviceCanAccessPeer(&can, p->device, root_device) == hipSuccess && can) {
				hipError_t e = hipDeviceEnablePeerAccess(root_device, 0);
				if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(MBIK_EHIP, "hipDeviceEnablePeerAccess");
				(void)hipGetLastError();
				DeviceGuard r(root_device);
				e = hipDeviceEnablePeerAccess(p->device, 0);
				if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(MBIK_EHIP, "hipDeviceEnablePeerAccess");
				(void)hipGetLastError();
			}
		}
		const size_t n = (size_t)p->host.N;
		if (hipMalloc(&s.in, std::max<size_t>(1, n * B * 10) * sizeof(float)) != hipSuccess ||
				hipMalloc(&s.tg, std::max<size_t>(1, n * P * 12) * sizeof(float)) != hipSuccess ||
				hipMalloc(&s.out, std::max<size_t>(1, n * B * 10) * sizeof(float)) != hipSuccess)
			return fail(MBIK_ENOMEM, "hipMalloc multi staging");
	}
	*out = m.release();
	return MBIK_OK;
}

int64_t mbik_multi_skeletons(const mbik_multi *m, int64_t *off) {
	if (!m) return fail(MBIK_EINVAL, "null handle");
	if (off) std::copy(m->off.begin(), m->off.end(), off);
	return m->off.back();
}

int32_t mbik_multi_solve(mbik_multi *m, const float *pose_in, const float *targets, float *pose_out, void *root_stream) {
	if (!m) return fail(MBIK_EINVAL, "null handle");
	if (!pose_in || !pose_out || (m->plans[0]->host.P > 0 && !targets)) return fail(MBIK_EINVAL, "null buffer");
	const int B = m->plans[0]->host.B, P = m->plans[0]->host.P;
	hipStream_t rs = reinterpret_cast<hipStream_t>(root_stream);
	{
		DeviceGuard g(m->root);
		if (hipEventRecord(m->start, rs) != hipSuccess) return fail(MBIK_EHIP, "hipEventRecord");
	}
	// Shards run in order; a failing shard ends the call.  Every shard that queued anything --
	// the failing one included -- records its done event on its stream, and the root stream waits
	// for all of those: the scatter copies still reading the caller's pose_in / targets and the
	// gathers writing pose_out finish before any later work on the root stream.
	int rc = MBIK_OK;
	size_t queued = 0;
	for (size_t i = 0; i < m->plans.size() && rc == MBIK_OK; i++) {
		mbik_plan *p = m->plans[i];
		auto &s = m->sh[i];
		const int64_t o = m->off[i];
		const size_t n = (size_t)p->host.N;
		DeviceGuard g(p->device);
		if (hipStreamWaitEvent(s.stream, m->start, 0) != hipSuccess) {
			rc = fail(MBIK_EHIP, "hipStreamWaitEvent");
			break;
		}
		queued = i + 1;
		const float *in = pose_in + o * B * 10, *tg = targets ? targets + o * P * 12 : nullptr;
		float *outp = pose_out + o * B * 10;
		if (s.staged && n) {
			if (hipMemcpyPeerAsync(s.in, p->device, in, m->root, n * B * 10 * sizeof(float), s.stream) != hipSuccess ||
					(P > 0 && hipMemcpyPeerAsync(s.tg, p->device, tg, m->root, n * P * 12 * sizeof(float), s.stream) != hipSuccess))
				rc = fail(MBIK_EHIP, "hipMemcpyPeerAsync (scatter)");
			else if ((rc = mbik_solve(p, 0, (int32_t)n, s.in, s.tg, s.out, s.stream)) != MBIK_OK)
				;
			else if (hipMemcpyPeerAsync(outp, m->root, s.out, p->device, n * B * 10 * sizeof(float), s.stream) != hipSuccess)
				rc = fail(MBIK_EHIP, "hipMemcpyPeerAsync (gather)");
		} else if (n) {
			rc = mbik_solve(p, 0, (int32_t)n, in, tg, outp, s.stream);
		}
		if (hipEventRecord(s.done, s.stream) != hipSuccess && rc == MBIK_OK) rc = fail(MBIK_EHIP, "hipEventRecord");
	}
	DeviceGuard g(m->root);
	for (size_t i = 0; i < queued; i++)
		if (hipStreamWaitEvent(rs, m->sh[i].done, 0) != hipSuccess && rc == MBIK_OK) rc = fail(MBIK_EHIP, "hipStreamWaitEvent");
	return rc;
}

} // extern "C"
