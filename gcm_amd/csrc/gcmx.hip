// gcmx.hip -- the C-ABI (include/gcmx.h): device contexts, layout transforms,
// per-tau stage tables, kernel-path selection, RCCL X-slab halo exchange and
// per-kernel event timing.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gcmx.h"
#include "common.hpp"
#include "launch.hpp"

using namespace gcmx;
static_assert(GCMX_MAX_BORDER_Q == kMaxBorderQ, "border quantity limit");
static_assert(GCMX_MAX_FACE_CONDITIONS == kMaxFaceConds && GCMX_NO_FACE_CONDITION == kNoFaceCond, "face maps");

namespace {

thread_local std::string g_last_error;

gcmx_status fail(gcmx_status s, const std::string& msg) {
	g_last_error = msg;
	return s;
}

}  // namespace

namespace gcmx {
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace gcmx

namespace {

#define HIP_TRY(expr)                                                                   \
	do {                                                                                \
		hipError_t e_ = (expr);                                                         \
		if (e_ != hipSuccess)                                                           \
			return fail(GCMX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
	} while (0)

struct PendingTiming {
	int bucket;
	double bytes;
	hipEvent_t a, b;
};

struct Bucket {
	std::string name;
	double total_ms = 0;
	long long launches = 0;
	double bytes = 0;    // algorithmic bytes summed over all timed launches
	std::string kernel;  // the instance the last launch of the bucket ran
};

}  // namespace

// In-process slab group (gcmx_comm_init_local): the RCCL exchange's semantics
// with device copies.  Rank r posts generation g of its current layer (event
// `ready` recorded after the work that produced it); the second rank of each
// adjacent pair to post g issues that pair's two copies on its own comm stream,
// after both ranks' `ready` events, and records `done`; a rank's wait for g
// (host: until both its pairs were issued, then stream waits on their `done`)
// covers the copies INTO its ghost planes and OUT OF its inner planes, as an
// RCCL group's completion does.  Two event slots (g & 1) suffice: a rank's
// wait(g) precedes its post(g + 1), and pair g + 2 needs both posts of g + 2.
struct LocalComm {
	int n = 0;
	std::vector<gcmx_ctx*> ctx;
	std::mutex mu;
	std::condition_variable cv;
	std::vector<long long> posted;         // [rank]: posts made
	std::vector<long long> issued;         // [pair]: generations issued (pair i = ranks i, i+1)
	std::vector<int> issuer[2];            // [slot][pair]: 0 = rank i issued, 1 = rank i+1
	std::vector<double*> layer[2];         // [slot][rank]: the layer posted
	std::vector<hipEvent_t> ready[2];      // [slot][rank] (rank's device)
	std::vector<hipEvent_t> done[2][2];    // [slot][side][pair] (the issuing rank's device)
	bool aborted = false;
	std::string why;
	~LocalComm() {
		for (int t = 0; t < 2; t++) {
			for (hipEvent_t e : ready[t])
				if (e) (void)hipEventDestroy(e);
			for (int sd = 0; sd < 2; sd++)
				for (hipEvent_t e : done[t][sd])
					if (e) (void)hipEventDestroy(e);
		}
	}
};

// A virtual range backed by physical chunks (vmm_map): its base, size and the
// chunks' handles in mapping order (empty: not in use).
struct VmmBlock {
	void* va = nullptr;
	size_t bytes = 0;
	std::vector<hipMemGenericAllocationHandle_t> chunks;
	unsigned long long granted = 0;  // devices given read-write access (bit d; the owner's at mapping)
};

struct gcmx_ctx {
	int device = 0;
	hipStream_t stream = nullptr;
	hipStream_t comm_stream = nullptr;
	hipStream_t inner_stream = nullptr;  // interior planes of the X-slab schedule (low priority)
	hipStream_t bnd_stream = nullptr;    // right boundary planes of the X-slab schedule
	hipEvent_t ev_ready = nullptr, ev_halo = nullptr;
	hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_bnd = nullptr;
	gcmx_grid_desc desc{};
	Geo geo{};
	int D = 0, M = 0, bs = 0;
	long long n_all = 0;         // reference all-nodes count
	long long all_shape[3] = {1, 1, 1};
	size_t layer_elems = 0;      // M * cs
	double* cur = nullptr;
	double* nxt = nullptr;
	double* layer_a = nullptr;   // the two layers as allocated (cur / nxt swap every step)
	double* layer_b = nullptr;
	void* layers_block = nullptr;  // both layers in one allocation (GCMX_LAYER_GAP), else null
	// layers_block mapped from physical chunks in shuffled order (vmm_map); empty
	// when hipMalloc'd
	VmmBlock vmm;
	// gcmx_layer_info out[3]: 0 two allocations, 1 one hipMalloc'd block, 2 one
	// physically contiguous block, else the shuffled mapping's chunk bytes
	uint64_t alloc_kind = 0;
	// clock sampler (gcmx_clock_probe_*): its own stream and sample buffer
	hipStream_t probe_stream = nullptr;
	unsigned long long* probe_d = nullptr;
	int probe_cap = 0;
	// materials
	int n_mat = 0;
	std::vector<double> U, U1, L;  // [mat][D][M*M], [mat][D][M]
	uint8_t* mat_d = nullptr;      // inner nodes, linear inner order; null = homogeneous
	int max_mat_id = -1;           // largest id in mat_d (set_materials must cover it)
	AxisTable* tabs_d = nullptr;   // [mat][D]
	double tabs_tau = NAN;
	bool iso_fast = false;         // fast kernels admissible (3-D, homogeneous, iso structure)
	bool iso2_fast = false;        // the 2-D one-pass step may run its isotropic kernel
	IsoAxis iso[3] = {};           // per-axis values for the fast kernels (tau part in build_tables)
	bool iso_het = false;          // per-node materials, every material of the iso structure (k_step_tx2 HET)
	bool het_ok = false;           // this tau: floor(q) = 0 and equal axes for every material
	std::vector<IsoAxis> het_iso;  // [mat]: tau-independent part (axis 0)
	IsoAxis* het_d = nullptr;      // [mat] on the device, per tau
	bool ghosts_touched = false;   // node-list border fills / contact copies / ghost uploads happened
	bool last_ode_fused = false;   // the last gcmx_step_ode scaled the stresses in the step's epilogue
	unsigned faces_written = 0;    // faces (bit 2*axis + side) whose ghosts a face fill wrote
	gcmx_path path = GCMX_PATH_AUTO;
	gcmx_schedule sched = GCMX_SCHED_AUTO;
	gcmx_path last_path = GCMX_PATH_AUTO;  // what the last step / stage ran
	int rows_per_block = 0;        // fused kernel y rows per block (0 = automatic)
	gcmx_fp_mode fp_mode = GCMX_FP_FMA;  // one-pass step build: contracted (default) or exact
	// halo exchange
	ncclComm_t comm = nullptr;
	bool comm_dead = false;         // the communicator failed and was aborted: every exchange fails
	bool comm_stall = false;        // tests only (gcmx_comm_test_stall): post sends, never receives
	double comm_timeout_s = 60.0;   // bound of every host wait on RCCL work
	int channels_per_peer = -1;     // NCCL_NCHANNELS_PER_PEER in effect (0: RCCL's default)
	long long halo_posted_calls = 0;  // ncclSend + ncclRecv calls posted (gcmx_comm_posted_calls)
	int nranks = 1, rank = 0, left = -1, right = -1;
	bool halo_pending = false;     // an exchange is in flight on comm_stream (ev_halo)
	bool step_posted = false;      // the current step posted its new boundary planes already
	bool halo_fresh = false;       // the current layer's ghost planes hold its neighbours' planes
	double* halo_layer = nullptr;  // the layer the pending exchange fills
	std::vector<int> halo_comps;
	std::shared_ptr<LocalComm> lc;  // in-process slab group (gcmx_comm_init_local)
	bool loop = false;              // loopback transport (gcmx_comm_init_loopback)
	double loop_gbps = 0;           // emulated link rate per direction (0: no hold)
	int loop_blocks = 0;            // blocks of the loopback copy kernel
	int lrank = -1;
	long long halo_gen = 0;        // posts made (in-process group)
	// profiling
	bool prof = false;
	std::vector<Bucket> buckets;
	std::vector<PendingTiming> pending;
	std::vector<hipEvent_t> event_pool;  // recycled timing events (no create/destroy per launch)
	// scratch for gcmx_border_fill (the node list of one call)
	int* nodes_d = nullptr;
	size_t nodes_cap = 0;
	double* ode_d = nullptr;  // per-material ODE factors (256)
};

struct gcmx_border_nodes {
	gcmx_ctx* ctx = nullptr;
	int axis = 0, side = 0, n = 0;
	int* nodes_d = nullptr;
};

// Per-node conditions of a body's faces (gcmx_face_map_create): one byte per
// face node, the index of the last condition whose area holds it or
// kNoFaceCond; the conditions' tables are written on the stream every step.
struct gcmx_face_map {
	gcmx_ctx* ctx = nullptr;
	uint8_t* map_d[6] = {};  // per-node conditions of a face that mixes them
	int uni[6] = {-1, -1, -1, -1, -1, -1};  // a face whose every node has condition uni[f]: no map
	unsigned used[6] = {};  // per face: bit k = condition k occurs on it
	BorderQ* bq_d = nullptr;
	FaceCond* fc_d = nullptr;
};

namespace {

int bucket_id(gcmx_ctx* c, const char* name) {
	for (size_t i = 0; i < c->buckets.size(); i++)
		if (c->buckets[i].name == name) return (int)i;
	c->buckets.push_back(Bucket{name});
	return (int)c->buckets.size() - 1;
}

hipEvent_t take_event(gcmx_ctx* c) {
	hipEvent_t ev = nullptr;
	if (!c->event_pool.empty()) {
		ev = c->event_pool.back();
		c->event_pool.pop_back();
	} else {
		(void)hipEventCreate(&ev);
	}
	return ev;
}

// Bracket one launch with events when profiling.
struct Timed {
	gcmx_ctx* c;
	int b;
	double bytes;
	hipEvent_t a = nullptr, e = nullptr;
	hipStream_t st;
	const char* kname = nullptr;  // set by the launcher: the instance it ran
	Timed(gcmx_ctx* c_, const char* name, double bytes_, hipStream_t s)
	    : c(c_), b(-1), bytes(bytes_), st(s) {
		if (!c->prof) return;
		b = bucket_id(c, name);
		a = take_event(c);
		e = take_event(c);
		(void)hipEventRecord(a, st);
	}
	~Timed() {
		if (b < 0) return;
		(void)hipEventRecord(e, st);
		c->pending.push_back({b, bytes, a, e});
		if (kname) c->buckets[b].kernel = kname;
	}
};

void drain_timings(gcmx_ctx* c) {
	for (auto& p : c->pending) {
		float ms = 0;
		(void)hipEventSynchronize(p.b);
		(void)hipEventElapsedTime(&ms, p.a, p.b);
		c->buckets[p.bucket].total_ms += ms;
		c->buckets[p.bucket].launches += 1;
		c->buckets[p.bucket].bytes += p.bytes;
		c->event_pool.push_back(p.a);
		c->event_pool.push_back(p.b);
	}
	c->pending.clear();
}

long long round_up(long long v, long long m) { return (v + m - 1) / m * m; }

// GCMX_ROW_PAD and friends (gcmx_create): a non-negative element count rounded
// up to `align`; 0 when unset.
static long long layout_pad(const char* name, long long align) {
	const char* e = std::getenv(name);
	const long long v = (e && *e) ? std::atoll(e) : 0;
	return v > 0 ? round_up(v, align) : 0;
}

// Element offset (device layout) of node `it` (multi-index incl. ghosts).
long long dev_offset(const Geo& g, const int it[3]) {
	long long o = g.origin;
	for (int d = 0; d < g.D; d++) o += (long long)it[d] * g.stride[d];
	return o;
}

gcmx_status check_ctx(gcmx_ctx* c) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null context");
	if (hipSetDevice(c->device) != hipSuccess) return fail(GCMX_ERR_HIP, "hipSetDevice failed");
	return GCMX_OK;
}

// Per-tau tables: crossingPoints (GridCharacteristicMethod.hpp:56-59), q = |dx|/h
// (:84), k = floor(q) with the reference's interpolation assertions
// (EqualDistanceLineInterpolator.hpp:20-23) and the Newton coefficients (:58-66).
gcmx_status build_tables(gcmx_ctx* c, double tau) {
	if (c->n_mat <= 0) return fail(GCMX_ERR_STATE, "materials not set");
	if (std::memcmp(&tau, &c->tabs_tau, sizeof(double)) == 0) return GCMX_OK;
	const int D = c->D, M = c->M, bs = c->bs;
	std::vector<AxisTable> h((size_t)c->n_mat * D);
	for (int m = 0; m < c->n_mat; m++)
		for (int s = 0; s < D; s++) {
			AxisTable& t = h[(size_t)m * D + s];
			std::memset(&t, 0, sizeof(t));
			const double* Um = &c->U[((size_t)m * D + s) * M * M];
			const double* U1m = &c->U1[((size_t)m * D + s) * M * M];
			const double* Lm = &c->L[((size_t)m * D + s) * M];
			for (int i = 0; i < M * M; i++) {
				t.U[i] = Um[i];
				t.U1[i] = U1m[i];
			}
			for (int k = 0; k < M; k++) {
				const double dx = Lm[k] * (-tau);
				const double q = std::fabs(dx) / c->desc.h[s];
				if (!(q >= 0))
					return fail(GCMX_ERR_CFL, "interpolation point q < 0 (reference assert_ge)");
				const double kf = std::floor(q);
				if (!(kf < bs)) {
					char buf[256];
					std::snprintf(buf, sizeof buf,
					              "Courant too large: q = %.17g >= borderSize %d on axis %d "
					              "(reference assert in minMaxInterpolate)", q, bs, s);
					return fail(GCMX_ERR_CFL, buf);
				}
				t.shift[k] = (dx > 0) ? 1 : -1;
				t.kf[k] = (int)kf;
				t.zero_q[k] = (q == 0) ? 1 : 0;
				for (int i = 1; i <= bs; i++) t.coef[k][i - 1] = ((q - i) + 1) / i;
			}
		}
	if (c->iso_fast || c->iso2_fast) {
		const int nfeet = D == 3 ? 6 : 4;
		for (int s = 0; s < D; s++) {
			const AxisTable& t = h[s];
			IsoAxis& A = c->iso[s];
			// feet k and k^1 share q; feet 2..5 (2-D: 2, 3) share q (|L| equal, checked at extraction)
			for (int k = 1; k < nfeet; k++) {
				const int ref = (k < 2) ? 0 : 2;
				if (t.kf[k] != t.kf[ref] || std::memcmp(t.coef[k], t.coef[ref], sizeof(t.coef[k])) != 0)
					return fail(GCMX_ERR_STATE, "inconsistent foot data");
			}
			for (int i = 0; i < 3; i++) {
				A.c1[i] = i < bs ? t.coef[0][i] : 0.0;
				A.c2[i] = i < bs ? t.coef[2][i] : 0.0;
			}
			A.kf1 = t.kf[0];
			A.kf2 = t.kf[2];
			lagrange_weights(A.c1, A.kf1 == 0 ? bs : 0, A.w1);
			lagrange_weights(A.c2, A.kf2 == 0 ? bs : 0, A.w2);
		}
	}
	HIP_TRY(hipMemcpyAsync(c->tabs_d, h.data(), h.size() * sizeof(AxisTable),
	                       hipMemcpyHostToDevice, c->stream));
	if (c->iso_het) {
		// one IsoAxis per material for all three stages: the axes' tables must be
		// bitwise equal (equal h) and every foot in [node, node + 1) (floor(q) = 0)
		std::vector<IsoAxis> ht(c->n_mat);
		bool ok = true;
		for (int m = 0; m < c->n_mat && ok; m++) {
			IsoAxis A[3];
			for (int s = 0; s < 3 && ok; s++) {
				const AxisTable& t = h[(size_t)m * D + s];
				ok = iso_axis_extract(s, &c->U[((size_t)m * D + s) * M * M], &c->U1[((size_t)m * D + s) * M * M],
				                      &c->L[((size_t)m * D + s) * M], A[s]);
				for (int k = 1; k < 6 && ok; k++) {
					const int ref = (k < 2) ? 0 : 2;
					ok = t.kf[k] == t.kf[ref] && std::memcmp(t.coef[k], t.coef[ref], sizeof(t.coef[k])) == 0;
				}
				for (int i = 0; i < 3; i++) {
					A[s].c1[i] = i < bs ? t.coef[0][i] : 0.0;
					A[s].c2[i] = i < bs ? t.coef[2][i] : 0.0;
				}
				A[s].kf1 = t.kf[0];
				A[s].kf2 = t.kf[2];
				lagrange_weights(A[s].c1, A[s].kf1 == 0 ? bs : 0, A[s].w1);
				lagrange_weights(A[s].c2, A[s].kf2 == 0 ? bs : 0, A[s].w2);
				ok = ok && A[s].kf1 == 0 && A[s].kf2 == 0;
			}
			ok = ok && std::memcmp(&A[0], &A[1], sizeof(IsoAxis)) == 0 && std::memcmp(&A[0], &A[2], sizeof(IsoAxis)) == 0;
			ht[m] = A[0];
		}
		c->het_ok = ok;
		if (ok) {
			if (!c->het_d) HIP_TRY(hipMalloc(&c->het_d, 256 * sizeof(IsoAxis)));
			HIP_TRY(hipMemcpyAsync(c->het_d, ht.data(), ht.size() * sizeof(IsoAxis), hipMemcpyHostToDevice,
			                       c->stream));
		}
	}
	HIP_TRY(hipStreamSynchronize(c->stream));
	c->tabs_tau = tau;
	return GCMX_OK;
}

// Components the X stage reads at the neighbours (those to put in the halo).
void compute_halo_comps(gcmx_ctx* c) {
	const int D = c->D, M = c->M;
	c->halo_comps.clear();
	for (int j = 0; j < M; j++) {
		bool need = false;
		for (int m = 0; m < c->n_mat && !need; m++)
			for (int k = 0; k < M && !need; k++) {
				const double Lk = c->L[((size_t)m * D + 0) * M + k];
				if (Lk != 0.0 && c->U[(((size_t)m * D + 0) * M + k) * M + j] != 0.0) need = true;
			}
		if (need) c->halo_comps.push_back(j);
	}
}

bool has_halo(const gcmx_ctx* c) {
	return (c->comm || c->comm_dead || c->lc || c->loop) && (c->left >= 0 || c->right >= 0);
}

// Bound of host waits on RCCL work: GCMX_COMM_TIMEOUT_SECONDS, default 60.
double comm_timeout_seconds() {
	const char* e = std::getenv("GCMX_COMM_TIMEOUT_SECONDS");
	const double d = e ? std::atof(e) : 0.0;
	return d > 0 ? d : 60.0;
}

// The communicator failed: abort it (RCCL's kernels waiting on a peer exit, so
// the streams drain), keep the context unable to exchange, report GCMX_ERR_COMM.
gcmx_status comm_fail(gcmx_ctx* c, const std::string& msg) {
	if (c->comm) (void)ncclCommAbort(c->comm);
	c->comm = nullptr;
	c->comm_dead = true;
	c->halo_pending = false;
	c->halo_fresh = false;
	return fail(GCMX_ERR_COMM, msg);
}

// Non-blocking communicator: wait (bounded) until its last call has completed
// its host part (ncclCommGetAsyncError leaves ncclInProgress).
gcmx_status comm_settle(gcmx_ctx* c, const char* what) {
	const auto t0 = std::chrono::steady_clock::now();
	for (long it = 0;; it++) {
		ncclResult_t st = ncclSuccess;
		const ncclResult_t r = ncclCommGetAsyncError(c->comm, &st);
		if (r != ncclSuccess) return comm_fail(c, std::string(what) + ": ncclCommGetAsyncError: " + ncclGetErrorString(r));
		if (st == ncclSuccess) return GCMX_OK;
		if (st != ncclInProgress) return comm_fail(c, std::string(what) + ": " + ncclGetErrorString(st));
		const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		if (el > c->comm_timeout_s)
			return comm_fail(c, std::string(what) + ": no progress within " + std::to_string(c->comm_timeout_s) +
			                        " s (a peer missing or dead?); communicator aborted");
		if (it > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
	}
}

// Host wait for a stream.  With an RCCL communicator the stream may depend on a
// peer (the exchange, or a compute stream waiting for it), so the wait polls
// under the communicator's timeout and its async error; a stalled exchange
// aborts the communicator (its kernels then exit and the stream drains) and
// returns GCMX_ERR_COMM instead of hanging.
gcmx_status wait_stream(gcmx_ctx* c, hipStream_t st, const char* what) {
	if (!c->comm) {
		HIP_TRY(hipStreamSynchronize(st));
		return GCMX_OK;
	}
	const auto t0 = std::chrono::steady_clock::now();
	for (long it = 0;; it++) {
		const hipError_t q = hipStreamQuery(st);
		if (q == hipSuccess) return GCMX_OK;
		if (q != hipErrorNotReady) return fail(GCMX_ERR_HIP, std::string(what) + ": " + hipGetErrorString(q));
		ncclResult_t as = ncclSuccess;
		if (ncclCommGetAsyncError(c->comm, &as) == ncclSuccess && as != ncclSuccess && as != ncclInProgress) {
			gcmx_status s = comm_fail(c, std::string(what) + ": RCCL async error: " + ncclGetErrorString(as));
			(void)hipStreamSynchronize(st);
			return s;
		}
		const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		if (el > c->comm_timeout_s) {
			gcmx_status s = comm_fail(c, std::string(what) + ": the halo exchange did not complete within " +
			                                 std::to_string(c->comm_timeout_s) +
			                                 " s (a peer missing or dead?); communicator aborted");
			(void)hipStreamSynchronize(st);  // the aborted RCCL kernels exit
			return s;
		}
		if (it > 256) std::this_thread::sleep_for(std::chrono::microseconds(100));
	}
}

// The current layer changed: its ghost planes no longer hold the neighbours' planes.
void touch_layer(gcmx_ctx* c) { c->halo_fresh = false; }

// x-plane x (all y/z rows including ghosts and row padding) of component `comp`
// of `layer`: for D >= 2 the contiguous range [(x + bs) * stride0, (x + bs + 1) * stride0).
double* plane_ptr(const gcmx_ctx* c, double* layer, int comp, int x) {
	return layer + (size_t)comp * c->geo.cs + (size_t)((long long)(x + c->bs) * c->geo.stride[0]);
}

// How long a rank waits for a neighbour's post: GCMX_LOCAL_WAIT_SECONDS, default 60.
double local_wait_seconds() {
	const char* e = std::getenv("GCMX_LOCAL_WAIT_SECONDS");
	const double d = e ? std::atof(e) : 0.0;
	return d > 0 ? d : 60.0;
}

// In-process group: post generation halo_gen of the current layer.
gcmx_status local_post(gcmx_ctx* c) {
	LocalComm& L = *c->lc;
	const int r = c->lrank;
	const long long g = c->halo_gen;
	const int slot = (int)(g & 1);
	HIP_TRY(hipEventRecord(L.ready[slot][r], c->stream));
	std::unique_lock<std::mutex> lk(L.mu);
	if (L.aborted) return fail(GCMX_ERR_COMM, "in-process slab group aborted: " + L.why);
	L.layer[slot][r] = c->cur;
	L.posted[r] = g + 1;
	for (int pr = r - 1; pr <= r; pr++) {  // pairs (r-1, r) and (r, r+1)
		if (pr < 0 || pr + 1 >= L.n) continue;
		const int other = (pr == r) ? r + 1 : r - 1;
		if (L.posted[other] != g + 1) continue;  // the other rank issues this pair
		gcmx_ctx* a = L.ctx[pr];
		gcmx_ctx* b = L.ctx[pr + 1];
		HIP_TRY(hipStreamWaitEvent(c->comm_stream, L.ready[slot][r], 0));
		HIP_TRY(hipStreamWaitEvent(c->comm_stream, L.ready[slot][other], 0));
		double* la = L.layer[slot][pr];
		double* lb = L.layer[slot][pr + 1];
		const size_t bytes = (size_t)(c->bs * c->geo.stride[0]) * sizeof(double);
		const int Xa = a->geo.sizes[0];
		for (int comp : c->halo_comps) {
			// a's right ghosts [Xa, Xa+bs) <- b's inner [0, bs); b's left ghosts [-bs, 0) <- a's inner [Xa-bs, Xa)
			HIP_TRY(hipMemcpyPeerAsync(plane_ptr(a, la, comp, Xa), a->device, plane_ptr(b, lb, comp, 0), b->device,
			                           bytes, c->comm_stream));
			HIP_TRY(hipMemcpyPeerAsync(plane_ptr(b, lb, comp, -b->bs), b->device, plane_ptr(a, la, comp, Xa - a->bs),
			                           a->device, bytes, c->comm_stream));
		}
		const int side = (r == pr) ? 0 : 1;
		HIP_TRY(hipEventRecord(L.done[slot][side][pr], c->comm_stream));
		L.issuer[slot][pr] = side;
		L.issued[pr] = g + 1;
	}
	lk.unlock();
	L.cv.notify_all();
	c->halo_gen = g + 1;
	return GCMX_OK;
}

// In-process group: wait for the last posted generation (both pairs issued).
gcmx_status local_wait(gcmx_ctx* c) {
	LocalComm& L = *c->lc;
	const int r = c->lrank;
	const long long g = c->halo_gen - 1;
	const int slot = (int)(g & 1);
	std::unique_lock<std::mutex> lk(L.mu);
	auto issued = [&] {
		for (int pr = r - 1; pr <= r; pr++)
			if (pr >= 0 && pr + 1 < L.n && L.issued[pr] < g + 1) return false;
		return true;
	};
	const double wait_s = local_wait_seconds();
	const bool ok = L.cv.wait_for(lk, std::chrono::duration<double>(wait_s),
	                              [&] { return L.aborted || issued(); });
	if (L.aborted) return fail(GCMX_ERR_COMM, "in-process slab group aborted: " + L.why);
	if (!ok)
		return fail(GCMX_ERR_COMM,
		            "in-process slab group: a neighbour did not post its halo within " +
		                std::to_string(wait_s) +
		                " s (the contexts must be stepped concurrently, one host thread each)");
	for (int pr = r - 1; pr <= r; pr++) {
		if (pr < 0 || pr + 1 >= L.n) continue;
		HIP_TRY(hipStreamWaitEvent(c->stream, L.done[slot][L.issuer[slot][pr]][pr], 0));
	}
	return GCMX_OK;
}

void local_abort(gcmx_ctx* c, const std::string& why) {
	if (!c || !c->lc) return;
	{
		std::lock_guard<std::mutex> lk(c->lc->mu);
		if (!c->lc->aborted) c->lc->why = why;
		c->lc->aborted = true;
	}
	c->lc->cv.notify_all();
}

// Loopback transport (gcmx_comm_init_loopback): ONE slab exchanging with itself
// periodically -- its right inner planes into its left ghost planes and its left
// inner planes into its right ghost planes, the halo components only -- by a
// few blocks on the comm stream (where RCCL's send/recv kernels run), each block
// holding its CU slot until `min_ticks` of the 100 MHz real-time counter have
// passed since it started: an xGMI transfer's duration and CU footprint on one
// GPU, so one rank's step schedule can be timed with the exchange in flight.
struct LoopPlan {
	long long src[2 * kMaxM], dst[2 * kMaxM];  // element offsets of the planes, per (comp, side)
	int n;                                     // (comp, side) pairs
	long long half;                            // double2 elements per plane group (bs planes)
};
__global__ __launch_bounds__(256) void k_loop_halo(double* __restrict__ layer, LoopPlan p,
                                                   unsigned long long min_ticks) {
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	// per (comp, side): eight independent 16-byte loads in flight per lane, then
	// their stores (32-bit indices: a group of bs planes is < 2^31 elements)
	constexpr int U = 8;
	const int stride = (int)(gridDim.x * blockDim.x), half = (int)p.half;
	for (int k = 0; k < p.n; k++) {
		const double2* __restrict__ src = reinterpret_cast<const double2*>(layer + p.src[k]);
		double2* __restrict__ dst = reinterpret_cast<double2*>(layer + p.dst[k]);
		for (int i0 = (int)(blockIdx.x * blockDim.x + threadIdx.x); i0 < half; i0 += U * stride) {
			double2 v[U];
#pragma unroll
			for (int u = 0; u < U; u++)
				if (i0 + u * stride < half) v[u] = src[i0 + u * stride];
#pragma unroll
			for (int u = 0; u < U; u++)
				if (i0 + u * stride < half) dst[i0 + u * stride] = v[u];
		}
	}
	if (threadIdx.x == 0) {
		for (int it = 0; it < (1 << 24); it++) {  // bounded: ~4 s at most
			if (__builtin_amdgcn_s_memrealtime() - t0 >= min_ticks) break;
			__builtin_amdgcn_s_sleep(8);
		}
	}
	__syncthreads();
}

gcmx_status loop_post(gcmx_ctx* c) {
	const Geo& g = c->geo;
	const int X = g.sizes[0], bs = c->bs;
	LoopPlan p{};
	const long long plane = (long long)bs * g.stride[0];
	for (int comp : c->halo_comps) {
		const long long base = (long long)comp * g.cs;
		p.src[p.n] = base + (long long)(X - bs + bs) * g.stride[0];  // inner [X-bs, X)
		p.dst[p.n++] = base;                                        // ghosts [-bs, 0)
		p.src[p.n] = base + (long long)bs * g.stride[0];             // inner [0, bs)
		p.dst[p.n++] = base + (long long)(X + bs) * g.stride[0];     // ghosts [X, X+bs)
	}
	p.half = plane / 2;
	if (p.half >= (1LL << 31) - (1LL << 24)) return fail(GCMX_ERR_UNSUPPORTED, "loopback: planes too large");
	const double bytes_dir = (double)c->halo_comps.size() * plane * sizeof(double);
	const unsigned long long ticks =
	    c->loop_gbps > 0 ? (unsigned long long)(bytes_dir / (c->loop_gbps * 1e9) * 1e8) : 0ull;
	HIP_TRY(hipEventRecord(c->ev_ready, c->stream));
	HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_ready, 0));
	{
		Timed t(c, "halo_loopback", 4.0 * bytes_dir, c->comm_stream);
		hipLaunchKernelGGL(k_loop_halo, dim3(c->loop_blocks), dim3(256), 0, c->comm_stream, c->cur, p, ticks);
		t.kname = "k_loop_halo";
	}
	HIP_TRY(hipGetLastError());
	HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
	c->halo_pending = true;
	c->halo_layer = c->cur;
	return GCMX_OK;
}

// Post the X-ghost exchange of the current layer on the comm stream (ordered
// after all work issued so far on the compute stream).  Completion is marked
// by ev_halo (RCCL) or the group's events (in-process); consumers call halo_wait.
gcmx_status halo_post(gcmx_ctx* c) {
	if (!has_halo(c)) return GCMX_OK;
	if (c->D < 2) return fail(GCMX_ERR_UNSUPPORTED, "X-slab halo needs dim >= 2");
	if (c->halo_comps.empty()) return fail(GCMX_ERR_STATE, "materials not set");
	if (c->lc) {
		gcmx_status s = local_post(c);
		if (s) return s;
		c->halo_pending = true;
		c->halo_layer = c->cur;
		return GCMX_OK;
	}
	if (c->loop) return loop_post(c);
	if (c->comm_dead || !c->comm) return fail(GCMX_ERR_COMM, "the communicator failed earlier and was aborted");
	const Geo& g = c->geo;
	const size_t n = (size_t)(c->bs * g.stride[0]);
	const int X = g.sizes[0];
	// ghost planes [-bs, 0) and [X, X+bs); inner planes [0, bs) and [X-bs, X).
	HIP_TRY(hipEventRecord(c->ev_ready, c->stream));
	HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_ready, 0));
	{
		// Profiling: the group on comm_stream, from the moment its data is ready
		// (the compute stream passed ev_ready) to its last kernel; bytes = what
		// this rank sends to ONE neighbour, i.e. what one link direction carries.
		Timed t(c, "halo_rccl", 8.0 * (double)n * (double)c->halo_comps.size(), c->comm_stream);
		t.kname = "ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd";
		ncclResult_t r = ncclGroupStart();
		if (r != ncclSuccess) return fail(GCMX_ERR_COMM, std::string("ncclGroupStart: ") + ncclGetErrorString(r));
		// Non-blocking communicator: a call may return ncclInProgress, which is
		// success so far; every later call of the group is still posted.  Every
		// failure inside the group still closes it (an open group would corrupt
		// every later call on the communicator).
		auto ok = [](ncclResult_t v) { return v == ncclSuccess || v == ncclInProgress; };
		std::string what;
		int posted = 0;
		for (int comp : c->halo_comps) {
			if (ok(r) && c->left >= 0) {
				what = "ncclSend/Recv left";
				r = ncclSend(plane_ptr(c, c->cur, comp, 0), n, ncclDouble, c->left, c->comm, c->comm_stream);
				posted += ok(r);
				if (ok(r) && !c->comm_stall) {
					r = ncclRecv(plane_ptr(c, c->cur, comp, -c->bs), n, ncclDouble, c->left, c->comm, c->comm_stream);
					posted += ok(r);
				}
			}
			if (ok(r) && c->right >= 0) {
				what = "ncclSend/Recv right";
				r = ncclSend(plane_ptr(c, c->cur, comp, X - c->bs), n, ncclDouble, c->right, c->comm, c->comm_stream);
				posted += ok(r);
				if (ok(r) && !c->comm_stall) {
					r = ncclRecv(plane_ptr(c, c->cur, comp, X), n, ncclDouble, c->right, c->comm, c->comm_stream);
					posted += ok(r);
				}
			}
		}
		const ncclResult_t re = ncclGroupEnd();
		if (!ok(r)) return comm_fail(c, what + ": " + ncclGetErrorString(r));
		if (!ok(re)) return comm_fail(c, std::string("ncclGroupEnd: ") + ncclGetErrorString(re));
		// every (component, neighbour) pair posted its send and, unless stalled on
		// purpose (tests), its receive: nothing of the group was skipped
		const int peers = (c->left >= 0) + (c->right >= 0);
		const int want = (int)c->halo_comps.size() * peers * (c->comm_stall ? 1 : 2);
		if (posted != want)
			return comm_fail(c, "halo exchange group: " + std::to_string(posted) + " of " + std::to_string(want) +
			                        " sends / receives posted");
		c->halo_posted_calls += posted;
		// non-blocking communicator: the group's kernels are on comm_stream once its
		// state leaves ncclInProgress; ev_halo must be recorded after them
		gcmx_status se = comm_settle(c, "halo exchange group");
		if (se) return se;
	}
	HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
	c->halo_pending = true;
	c->halo_layer = c->cur;
	return GCMX_OK;
}

gcmx_status halo_wait(gcmx_ctx* c) {
	if (!c->halo_pending) return GCMX_OK;
	{
		// Profiling: how long the compute stream stands still at this wait, i.e.
		// the part of the exchange that is NOT hidden behind compute (an event on
		// the stream before the wait, one after it)
		Timed t(c, "halo_wait", 0.0, c->stream);
		if (c->lc) {
			gcmx_status s = local_wait(c);
			if (s) return s;
		} else {
			HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
		}
	}
	c->halo_pending = false;
	c->halo_fresh = c->halo_layer == c->cur;
	return GCMX_OK;
}

gcmx_status halo_exchange_impl(gcmx_ctx* c) {
	gcmx_status s = halo_wait(c);  // an earlier exchange of this layer is still in flight
	if (s) return s;
	s = halo_post(c);
	if (s) return s;
	return halo_wait(c);
}

// Ghost planes of the current layer valid before an X stage reads them: the
// pending exchange, or a new one unless the layer's ghosts are already fresh.
gcmx_status halo_ensure(gcmx_ctx* c) {
	gcmx_status s = halo_wait(c);
	if (s || c->halo_fresh) return s;
	s = halo_post(c);
	if (s) return s;
	return halo_wait(c);
}

// Fast kernels: 3-D, one material, no per-node ids, isotropic zero pattern.
void refresh_fast(gcmx_ctx* c) {
	const int D = c->D, M = c->M;
	bool fits = (D == 3) && (c->mat_d == nullptr) && (c->n_mat == 1) && onepass_layout_ok(c->geo);
	for (int sx = 0; fits && sx < D; sx++)
		fits = iso_axis_extract(sx, &c->U[(size_t)sx * M * M], &c->U1[(size_t)sx * M * M],
		                        &c->L[(size_t)sx * M], c->iso[sx]);
	c->iso_fast = fits;
	// the 2-D one-pass step's isotropic kernel: one material, the ElasticModel<2> structure
	bool fits2 = D == 2 && c->mat_d == nullptr && c->n_mat == 1 && step2d_iso_supported(c->geo);
	for (int sx = 0; fits2 && sx < D; sx++)
		fits2 = iso2_axis_extract(sx, &c->U[(size_t)sx * M * M], &c->U1[(size_t)sx * M * M], &c->L[(size_t)sx * M],
		                          c->iso[sx]);
	c->iso2_fast = fits2;
	// heterogeneous one-pass step: per-node ids and every material of the structure
	bool het = !fits && D == 3 && c->mat_d != nullptr && c->n_mat >= 1 && c->n_mat <= kHetMaxMaterials &&
	           onepass_layout_ok(c->geo) && het_supported(c->geo);
	for (int m = 0; het && m < c->n_mat; m++)
		for (int sx = 0; het && sx < D; sx++) {
			IsoAxis tmp{};
			het = iso_axis_extract(sx, &c->U[((size_t)m * D + sx) * M * M], &c->U1[((size_t)m * D + sx) * M * M],
			                       &c->L[((size_t)m * D + sx) * M], tmp);
		}
	c->iso_het = het;
	c->het_ok = false;
	c->tabs_tau = NAN;
}

// The one-pass 2-D step (k_step2d) runs where its preconditions hold: one
// material, no ghost ever written (so every ghost of both layers is zero and
// the two layers' ghosts agree, whichever one the step leaves the state in),
// no X-slab exchange, a borderSize it is built for, and no forced per-stage path.
bool step2d_admissible(const gcmx_ctx* c) {
	return c->D == 2 && step2d_supported(c->geo) && c->mat_d == nullptr && c->n_mat == 1 && !c->ghosts_touched &&
	       c->faces_written == 0 && !has_halo(c) && c->path != GCMX_PATH_GENERIC && c->path != GCMX_PATH_SPLIT;
}
// The same with whole-face border conditions `on` (bit 2*axis + side): the
// isotropic kernel, the y ghost columns formed in the pass from the mirrored
// inner columns (Y >= bs + 1), and every face whose ghosts an earlier step wrote
// refreshed now.
bool step2d_faces_admissible(const gcmx_ctx* c, unsigned on) {
	return c->D == 2 && c->iso2_fast && step2d_iso_supported(c->geo) && c->mat_d == nullptr && c->n_mat == 1 &&
	       !c->ghosts_touched && (c->faces_written & ~on) == 0 && !has_halo(c) && c->path != GCMX_PATH_GENERIC &&
	       c->path != GCMX_PATH_SPLIT && c->geo.sizes[1] >= c->bs + 1;
}

gcmx_path effective_path(gcmx_ctx* c) {
	if (c->iso_het) {  // per-node materials: the one-pass step or the generic stages
		if (c->path == GCMX_PATH_GENERIC || c->path == GCMX_PATH_SPLIT || c->ghosts_touched) return GCMX_PATH_GENERIC;
		return GCMX_PATH_FUSED;
	}
	if (c->D == 2) return step2d_admissible(c) ? GCMX_PATH_FUSED : GCMX_PATH_GENERIC;
	if (c->D != 3 || !c->iso_fast || c->bs > 3) return GCMX_PATH_GENERIC;
	if (c->path == GCMX_PATH_GENERIC) return GCMX_PATH_GENERIC;
	// the per-stage kernels address whole layers with 32-bit offsets
	const gcmx_path split = fast_layout_ok(c->geo) ? GCMX_PATH_SPLIT : GCMX_PATH_GENERIC;
	if (c->path == GCMX_PATH_SPLIT) return split;
	if (c->ghosts_touched || !fused_supported(c->geo)) return split;
	return GCMX_PATH_FUSED;
}

double node_stage_bytes(const gcmx_ctx* c) { return 2.0 * c->M * sizeof(double); }

// PhysicalQuantities code -> component of the D-dimensional PDE vector
// (VelocitySigmaVariables.cpp:51-66); -1 if absent (PRESSURE: 12, handled apart).
int quantity_comp(int D, int q) {
	if (q >= 2 && q <= 4) return (q - 2) < D ? q - 2 : -1;
	if (q >= 5 && q <= 10) {
		static const int ii[6] = {0, 0, 0, 1, 1, 2}, jj[6] = {0, 1, 2, 1, 2, 2};
		const int i = ii[q - 5], j = jj[q - 5];
		if (i >= D || j >= D) return -1;
		return D + (i * D - ((i - 1) * i) / 2 + j - i);
	}
	return -1;
}

gcmx_status border_q(const gcmx_ctx* c, int n_q, const int* qs, const double* vals, BorderQ& bq) {
	if (n_q < 0 || n_q > kMaxBorderQ || (n_q > 0 && (!qs || !vals)))
		return fail(GCMX_ERR_INVALID_ARG, "bad border quantities (at most 16)");
	bq.n = n_q;
	for (int k = 0; k < n_q; k++) {
		if (qs[k] != 12 && quantity_comp(c->D, qs[k]) < 0)
			return fail(GCMX_ERR_INVALID_ARG, "quantity not in this PDE vector");
		bq.q[k] = qs[k];
		bq.v[k] = vals[k];
	}
	return GCMX_OK;
}

gcmx_status stage_impl(gcmx_ctx* c, int axis, double tau) {
	gcmx_status s = build_tables(c, tau);
	if (s != GCMX_OK) return s;
	s = halo_wait(c);
	if (s != GCMX_OK) return s;
	if (axis == 0 && has_halo(c)) {
		s = halo_ensure(c);
		if (s != GCMX_OK) return s;
	}
	const Geo& g = c->geo;
	const double bytes = node_stage_bytes(c) * (double)g.n_inner;
	// no per-stage het kernels; the per-stage kernels of the split path are 3-D only
	const gcmx_path p =
	    (c->iso_het || c->D != 3 || !fast_layout_ok(c->geo)) ? GCMX_PATH_GENERIC : effective_path(c);
	bool ok;
	if (p == GCMX_PATH_GENERIC) {
		Timed t(c, "stage_generic", bytes, c->stream);
		ok = launch_stage_generic(c->cur, c->nxt, g, axis, c->tabs_d, c->mat_d, c->stream);
		t.kname = "k_stage_generic";
	} else if (axis < 2) {
		Timed t(c, axis == 0 ? "march_x" : "march_y", bytes, c->stream);
		ok = launch_march(c->cur, c->nxt, g, axis, c->iso[axis], 0, g.sizes[0], c->stream);
		t.kname = axis == 0 ? "k_march<0>" : "k_march<1>";
	} else {
		Timed t(c, "line_z", bytes, c->stream);
		ok = launch_line_z(c->cur, c->nxt, g, c->iso[2], 0, g.sizes[0], c->stream);
		t.kname = "k_line_z";
	}
	if (!ok) return fail(GCMX_ERR_UNSUPPORTED, "no kernel variant for this configuration");
	HIP_TRY(hipGetLastError());
	std::swap(c->cur, c->nxt);
	touch_layer(c);
	c->last_path = p == GCMX_PATH_GENERIC ? GCMX_PATH_GENERIC : GCMX_PATH_SPLIT;
	return GCMX_OK;
}

}  // namespace

// =================================================================== ABI ==

extern "C" {

int gcmx_abi_version(void) { return GCMX_ABI_VERSION; }
const char* gcmx_last_error(void) { return g_last_error.c_str(); }
int gcmx_pde_size(int dim) { return (dim >= 1 && dim <= 3) ? pde_size(dim) : -1; }

const char* gcmx_status_string(gcmx_status s) {
	switch (s) {
	case GCMX_OK: return "ok";
	case GCMX_ERR_INVALID_ARG: return "invalid argument";
	case GCMX_ERR_CFL: return "Courant condition violated";
	case GCMX_ERR_HIP: return "HIP error";
	case GCMX_ERR_OOM: return "out of device memory";
	case GCMX_ERR_STATE: return "invalid call order";
	case GCMX_ERR_UNSUPPORTED: return "unsupported configuration";
	case GCMX_ERR_COMM: return "communication error";
	}
	return "unknown";
}

// Default chunk of the shuffled mapping (profiles/r5/r, s, t, u): 512^3 runs
// alike from 64 MiB to 1 GiB chunks (3.64-3.66 ms), 32 MiB and below lose
// (2 MiB: 4.80 ms); the 2-D 8192^2 block (5.4 GB) gains with 64 MiB chunks
// (1.11 against 1.27 ms) and not with 256 MiB ones; 256^3 and the N = 8 slab
// are alike with either.  256 MiB chunks for blocks of 8 GiB and more, 64 MiB below.
static long long shuffle_chunk_mib(size_t block) { return block >= (8ULL << 30) ? 256 : 64; }

// The layers' block as physical chunks of `chunk` bytes mapped into one
// virtual range in a shuffled order (HIP virtual memory management): whatever
// the physical free space looks like, consecutive virtual chunks land in
// unrelated physical places.  A large hipMalloc on a box whose VRAM is one free
// region comes back physically contiguous, and then the one-pass step's
// concurrent streams (9 components x 2*bs+2 planes x every CU's block) meet the
// HBM in a regular pattern: 512^3 4.14-4.17 ms from a contiguous block, 3.88-3.91
// where hipMalloc happened to scatter it, 3.58-3.65 ms from shuffled 64 MiB - 1 GiB
// chunks.  Returns false (nothing held) on failure.
static bool vmm_map(int device, size_t bytes, size_t chunk_req, VmmBlock& out) {
	hipMemAllocationProp prop{};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = device;
	size_t gran = 0;
	if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || gran == 0)
		return false;
	const size_t chunk = (chunk_req + gran - 1) / gran * gran;
	const size_t n = (bytes + chunk - 1) / chunk, total = n * chunk;
	void* va = nullptr;
	if (hipMemAddressReserve(&va, total, chunk, nullptr, 0) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	std::vector<hipMemGenericAllocationHandle_t> h;
	h.reserve(n);
	bool ok = true;
	for (size_t i = 0; i < n && ok; i++) {
		hipMemGenericAllocationHandle_t x{};
		ok = hipMemCreate(&x, chunk, &prop, 0) == hipSuccess;
		if (ok) h.push_back(x);
	}
	// a fixed pseudo-random permutation (Fisher-Yates over a 64-bit LCG)
	std::vector<size_t> perm(h.size());
	for (size_t i = 0; i < perm.size(); i++) perm[i] = i;
	unsigned long long st = 0x9E3779B97F4A7C15ULL;
	for (size_t i = perm.size(); i > 1; i--) {
		st = st * 6364136223846793005ULL + 1442695040888963407ULL;
		std::swap(perm[i - 1], perm[(size_t)((st >> 33) % i)]);
	}
	size_t mapped = 0;  // chunks mapped so far
	for (size_t i = 0; i < h.size() && ok; i++) {
		ok = hipMemMap(static_cast<char*>(va) + i * chunk, chunk, 0, h[perm[i]], 0) == hipSuccess;
		if (ok) mapped++;
	}
	if (ok) {
		hipMemAccessDesc a{};
		a.location = prop.location;
		a.flags = hipMemAccessFlagsProtReadWrite;
		ok = hipMemSetAccess(va, total, &a, 1) == hipSuccess;
	}
	if (!ok) {
		(void)hipGetLastError();
		for (size_t i = 0; i < mapped; i++) (void)hipMemUnmap(static_cast<char*>(va) + i * chunk, chunk);
		for (auto x : h) (void)hipMemRelease(x);
		(void)hipMemAddressFree(va, total);
		(void)hipGetLastError();
		return false;
	}
	out.va = va;
	out.bytes = total;
	out.chunks = std::move(h);
	out.granted = device < 64 ? 1ULL << device : 0;
	return true;
}

// Read-write access to a mapped block for another device (the in-process X-slab
// group copies between devices); false if the peer cannot be granted it.
// Granted once per (block, device): the grant walks the whole multi-GB mapping,
// so it is made at group set-up and cached, never per exchange.
static bool vmm_grant(VmmBlock& b, int peer) {
	if (!b.va) return true;
	const unsigned long long bit = peer >= 0 && peer < 64 ? 1ULL << peer : 0;
	if (bit && (b.granted & bit)) return true;
	hipMemAccessDesc a{};
	a.location.type = hipMemLocationTypeDevice;
	a.location.id = peer;
	a.flags = hipMemAccessFlagsProtReadWrite;
	if (hipMemSetAccess(b.va, b.bytes, &a, 1) == hipSuccess) {
		b.granted |= bit;
		return true;
	}
	(void)hipGetLastError();
	return false;
}

static void vmm_free(VmmBlock& b) {
	if (!b.va) return;
	const size_t chunk = b.bytes / b.chunks.size();
	for (size_t i = 0; i < b.chunks.size(); i++) (void)hipMemUnmap(static_cast<char*>(b.va) + i * chunk, chunk);
	for (auto x : b.chunks) (void)hipMemRelease(x);
	(void)hipMemAddressFree(b.va, b.bytes);
	b = VmmBlock{};
}

// The allocation policy of large device blocks (the layers, the copy-ceiling
// buffers): the shuffled mapping's chunk in MiB for a block of `block` bytes,
// 0 for none; `contig`: GCMX_ALLOC=contiguous.
static long long shuffle_policy_mib(size_t block, bool* contig) {
	static const long long env = [] {  // -1: the default rule, 0: no shuffling
		const char* e = std::getenv("GCMX_ALLOC");
		if (!e || !*e) return -1LL;
		if (std::strncmp(e, "shuffle:", 8) == 0) return std::max(1LL, std::atoll(e + 8));
		return 0LL;
	}();
	static const bool cont = [] {
		const char* e = std::getenv("GCMX_ALLOC");
		return e && std::strcmp(e, "contiguous") == 0;
	}();
	if (contig) *contig = cont;
	const long long mib = env < 0 ? shuffle_chunk_mib(block) : env;
	return (mib > 0 && block >= 2 * ((size_t)mib << 20)) ? mib : 0;
}

gcmx_status gcmx_create(const gcmx_grid_desc* d, int device, gcmx_ctx** out) {
	if (!d || !out) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	*out = nullptr;
	if (d->dim < 1 || d->dim > 3) return fail(GCMX_ERR_INVALID_ARG, "dim must be 1..3");
	// CubicGrid ctor: assert_gt(borderSize, 0), sizes >= borderSize, h > 0 (CubicGrid.hpp:193-199)
	if (d->border_size <= 0 || d->border_size > kMaxBs)
		return fail(GCMX_ERR_INVALID_ARG, "border_size must be 1..8");
	for (int i = 0; i < d->dim; i++) {
		if (d->sizes[i] < d->border_size)
			return fail(GCMX_ERR_INVALID_ARG, "sizes[i] must be >= border_size");
		if (!(d->h[i] > 0)) return fail(GCMX_ERR_INVALID_ARG, "h[i] must be > 0");
	}
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
		return fail(GCMX_ERR_HIP, "no HIP device available");
	if (device < 0 || device >= ndev) return fail(GCMX_ERR_INVALID_ARG, "bad device index");
	HIP_TRY(hipSetDevice(device));

	auto* c = new gcmx_ctx();
	c->device = device;
	// GCMX_FP=exact makes the exact build every new context's default (tests
	// that compare with the oracle bitwise); anything else keeps FMA.
	if (const char* e = std::getenv("GCMX_FP")) c->fp_mode = std::strcmp(e, "exact") == 0 ? GCMX_FP_EXACT : GCMX_FP_FMA;
	c->desc = *d;
	c->D = d->dim;
	c->M = pde_size(d->dim);
	c->bs = d->border_size;
	Geo& g = c->geo;
	g.D = c->D;
	g.M = c->M;
	g.bs = c->bs;
	const int D = c->D, bs = c->bs;
	for (int i = 0; i < 3; i++) g.sizes[i] = (i < D) ? d->sizes[i] : 1;
	g.gx0 = d->start[0];
	// fastest axis: `lead` unused elements, bs ghosts, inner, bs ghosts, padding
	const int last = D - 1;
	// Layout perturbation (tests only, GCMX_ROW_PAD / GCMX_PLANE_PAD / GCMX_CS_PAD:
	// extra elements per row, per 3-D x plane, per component plane, rounded to
	// keep the alignments): every kernel and host conversion must take its strides
	// from Geo, and tests/test_gpu_layout.py runs the suites' cases with the strides
	// no longer implied by the sizes.
	const long long row_pad = layout_pad("GCMX_ROW_PAD", kRowAlign);
	const long long plane_pad = D == 3 ? layout_pad("GCMX_PLANE_PAD", kRowAlign) : 0;
	const long long cs_pad = layout_pad("GCMX_CS_PAD", 64);
	g.lead = (int)round_up(bs, kRowAlign) - bs;
	g.row = round_up(g.lead + bs + d->sizes[last] + bs, kRowAlign) + row_pad;
	long long n_all_d[3] = {1, 1, 1};
	for (int i = 0; i < D; i++) n_all_d[i] = d->sizes[i] + 2LL * bs;
	for (int i = 0; i < 3; i++) g.stride[i] = 0;
	g.stride[last] = 1;
	long long st = g.row;
	for (int i = last - 1; i >= 0; i--) {
		g.stride[i] = st + (i == 0 ? plane_pad : 0);
		st = g.stride[i] * n_all_d[i];
	}
	const long long total = st;
	g.cs = round_up(total, 64) + cs_pad;
	g.origin = (long long)(g.lead + bs);  // fastest-axis offset of inner index 0
	for (int i = 0; i < last; i++) g.origin += (long long)bs * g.stride[i];
	g.n_inner = (long long)g.sizes[0] * g.sizes[1] * g.sizes[2];
	c->n_all = 1;
	for (int i = 0; i < D; i++) {
		c->all_shape[i] = n_all_d[i];
		c->n_all *= n_all_d[i];
	}
	c->layer_elems = (size_t)c->M * (size_t)g.cs;

	const size_t bytes = c->layer_elems * sizeof(double);
	// Layers: ONE allocation holding layer A, a 2 MiB gap, then layer B (both
	// 2 MiB-aligned: a layer is a whole number of 2 MiB fragments whenever its size
	// is).  Measured on one MI355X, fresh processes back to back (profiles/r4/swing):
	// the 512^3 step 4.198-4.200 ms with gaps of 0 / 4 KiB / 64 KiB / 2 MiB
	// against 4.243-4.259 ms for two separate allocations (nine processes) --
	// where the two layers lie relative to each other in HBM moves the streaming
	// step by ~1 %.  GCMX_LAYER_GAP = bytes (rounded to 256) sets the gap, < 0
	// gives two separate allocations (measurement only).
	long long gap = 2LL << 20;
	if (const char* e = std::getenv("GCMX_LAYER_GAP")) {
		const long long v = std::atoll(e);
		gap = v < 0 ? -1 : round_up(v, 256);
	}
	// Placement of the layers' block in physical memory (measured):
	// by default physical chunks (shuffle_chunk_mib) mapped in a shuffled order
	// (vmm_map) once the block spans two chunks; GCMX_ALLOC=malloc (one
	// hipMalloc), =contiguous (hipDeviceMallocContiguous) or =shuffle:<MiB>
	// chooses explicitly.  Any failure falls back to hipMalloc.
	bool alloc_ok;
	if (gap >= 0) {
		const size_t block = 2 * bytes + (size_t)gap;
		bool alloc_contig = false;
		const long long shuffle_mb = shuffle_policy_mib(block, &alloc_contig);
		alloc_ok = false;
		if (shuffle_mb > 0) {
			alloc_ok = vmm_map(c->device, block, (size_t)shuffle_mb << 20, c->vmm);
			if (alloc_ok) {
				c->layers_block = c->vmm.va;
				c->alloc_kind = c->vmm.bytes / c->vmm.chunks.size();
			} else {
				std::fprintf(stderr, "gcmx: shuffled chunk mapping failed, using hipMalloc\n");
			}
		}
		if (!alloc_ok && alloc_contig) {
			alloc_ok = hipExtMallocWithFlags(&c->layers_block, block, hipDeviceMallocContiguous) == hipSuccess;
			if (alloc_ok) {
				c->alloc_kind = 2;
			} else {
				(void)hipGetLastError();
				std::fprintf(stderr, "gcmx: contiguous allocation of %zu bytes failed, using hipMalloc\n", block);
			}
		}
		if (!alloc_ok) {
			alloc_ok = hipMalloc(&c->layers_block, block) == hipSuccess;
			c->alloc_kind = 1;
		}
		if (alloc_ok) {
			c->cur = static_cast<double*>(c->layers_block);
			c->nxt = reinterpret_cast<double*>(static_cast<char*>(c->layers_block) + bytes + (size_t)gap);
		}
	} else {
		alloc_ok = hipMalloc(&c->cur, bytes) == hipSuccess && hipMalloc(&c->nxt, bytes) == hipSuccess;
	}
	c->layer_a = c->cur;
	c->layer_b = c->nxt;
	if (!alloc_ok || hipMalloc(&c->tabs_d, sizeof(AxisTable) * 255 * 3) != hipSuccess) {
		gcmx_destroy(c);
		return fail(GCMX_ERR_OOM, "device allocation failed");
	}
	// Main stream at the highest priority, the interior-plane stream at the
	// lowest: the boundary planes of a slab step (and the halo they feed) are
	// dispatched ahead of the interior blocks that run beside them.
	// GCMX_STREAM_PRIO=normal (measurement only) gives every stream the default.
	int prio_lo = 0, prio_hi = 0;
	if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
	if (const char* e = std::getenv("GCMX_STREAM_PRIO"))
		if (std::strcmp(e, "normal") == 0) prio_lo = prio_hi = 0;
	if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
	    hipStreamCreateWithPriority(&c->inner_stream, hipStreamNonBlocking, prio_lo) != hipSuccess ||
	    hipStreamCreateWithPriority(&c->bnd_stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
	    hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
	    hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming) != hipSuccess ||
	    hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming) != hipSuccess ||
	    hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
	    hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
	    hipEventCreateWithFlags(&c->ev_bnd, hipEventDisableTiming) != hipSuccess) {
		gcmx_destroy(c);
		return fail(GCMX_ERR_HIP, "stream/event creation failed");
	}
	if (hipMemsetAsync(c->cur, 0, bytes, c->stream) != hipSuccess ||
	    hipMemsetAsync(c->nxt, 0, bytes, c->stream) != hipSuccess ||
	    hipStreamSynchronize(c->stream) != hipSuccess) {
		gcmx_destroy(c);
		return fail(GCMX_ERR_HIP, "zero fill failed");
	}
	*out = c;
	return GCMX_OK;
}

void gcmx_destroy(gcmx_ctx* c) {
	if (!c) return;
	(void)hipSetDevice(c->device);
	if (c->comm) {  // bounded: a stalled exchange aborts the communicator
		if (c->comm_stream) (void)wait_stream(c, c->comm_stream, "gcmx_destroy");
		if (c->stream && c->comm) (void)wait_stream(c, c->stream, "gcmx_destroy");
	}
	if (c->stream) (void)hipStreamSynchronize(c->stream);
	if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
	if (c->inner_stream) (void)hipStreamSynchronize(c->inner_stream);
	if (c->bnd_stream) (void)hipStreamSynchronize(c->bnd_stream);
	drain_timings(c);
	for (hipEvent_t ev : c->event_pool) (void)hipEventDestroy(ev);
	if (c->probe_stream) (void)hipStreamSynchronize(c->probe_stream);
	if (c->comm) {  // non-blocking communicator: finalize (bounded), then destroy; abort on failure
		ncclResult_t r = ncclCommFinalize(c->comm);
		if (r == ncclSuccess || r == ncclInProgress) {
			const std::string keep = g_last_error;
			if (comm_settle(c, "ncclCommFinalize") == GCMX_OK) (void)ncclCommDestroy(c->comm);
			g_last_error = keep;  // comm_settle aborted it on failure
		} else {
			(void)ncclCommAbort(c->comm);
		}
		c->comm = nullptr;
	}
	if (c->lc) {  // the group cannot exchange without this rank any more
		local_abort(c, "a context of the group was destroyed");
		std::lock_guard<std::mutex> lk(c->lc->mu);
		LocalComm& L = *c->lc;
		// A neighbour's comm stream may still copy into this rank's ghost planes or
		// out of its inner planes (pairs (r-1, r) and (r, r+1), either issuer, both
		// generation slots): wait for those copies before the layers are freed.
		for (int t = 0; t < 2; t++)
			for (int sd = 0; sd < 2; sd++)
				for (int pr = c->lrank - 1; pr <= c->lrank; pr++)
					if (pr >= 0 && pr < (int)L.done[t][sd].size() && L.done[t][sd][pr])
						(void)hipEventSynchronize(L.done[t][sd][pr]);
		L.ctx[c->lrank] = nullptr;
	}
	if (c->vmm.va) {
		// unmapping does not wait for the device (hipFree does): another context's
		// stream may still read these layers (gcmx_copy_box, an in-process group)
		(void)hipDeviceSynchronize();
		vmm_free(c->vmm);
	} else if (c->layers_block) {
		(void)hipFree(c->layers_block);
	} else {
		(void)hipFree(c->layer_a);
		(void)hipFree(c->layer_b);
	}
	(void)hipFree(c->probe_d);
	if (c->probe_stream) (void)hipStreamDestroy(c->probe_stream);
	(void)hipFree(c->tabs_d);
	(void)hipFree(c->mat_d);
	(void)hipFree(c->nodes_d);
	(void)hipFree(c->ode_d);
	(void)hipFree(c->het_d);
	if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
	if (c->ev_halo) (void)hipEventDestroy(c->ev_halo);
	if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
	if (c->ev_join) (void)hipEventDestroy(c->ev_join);
	if (c->ev_bnd) (void)hipEventDestroy(c->ev_bnd);
	if (c->stream) (void)hipStreamDestroy(c->stream);
	if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
	if (c->inner_stream) (void)hipStreamDestroy(c->inner_stream);
	if (c->bnd_stream) (void)hipStreamDestroy(c->bnd_stream);
	delete c;
}

gcmx_status gcmx_set_materials(gcmx_ctx* c, int n_mat, const double* U, const double* U1,
                               const double* L) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (n_mat < 1 || n_mat > 255 || !U || !U1 || !L)
		return fail(GCMX_ERR_INVALID_ARG, "n_mat must be 1..255 with non-null tables");
	// per-node ids set earlier index these tables (the device tables of the other
	// entries would be uninitialised)
	if (c->mat_d && c->max_mat_id >= n_mat)
		return fail(GCMX_ERR_INVALID_ARG, "material ids set earlier exceed the new material count");
	const int D = c->D, M = c->M;
	const size_t nm = (size_t)n_mat * D * M * M, nl = (size_t)n_mat * D * M;
	for (size_t i = 0; i < nm; i++)
		if (!std::isfinite(U[i]) || !std::isfinite(U1[i]))
			return fail(GCMX_ERR_INVALID_ARG, "non-finite matrix entry");
	for (size_t i = 0; i < nl; i++)
		if (!std::isfinite(L[i])) return fail(GCMX_ERR_INVALID_ARG, "non-finite eigenvalue");
	c->n_mat = n_mat;
	c->U.assign(U, U + nm);
	c->U1.assign(U1, U1 + nm);
	c->L.assign(L, L + nl);
	c->tabs_tau = NAN;
	refresh_fast(c);
	compute_halo_comps(c);
	return GCMX_OK;
}

gcmx_status gcmx_set_material_ids(gcmx_ctx* c, const uint8_t* ids) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!ids) {
		(void)hipFree(c->mat_d);
		c->mat_d = nullptr;
		c->max_mat_id = -1;
	} else {
		int mx = 0;
		const Geo& g = c->geo;
		std::vector<uint8_t> inner((size_t)g.n_inner);
		long long i = 0;
		for (int x = 0; x < g.sizes[0]; x++)
			for (int y = 0; y < g.sizes[1]; y++)
				for (int z = 0; z < g.sizes[2]; z++, i++) {
					const int it[3] = {x, y, z};
					long long ref = 0, mul = 1;
					for (int d = c->D - 1; d >= 0; d--) {
						ref += (it[d] + c->bs) * mul;
						mul *= c->all_shape[d];
					}
					const uint8_t m = ids[ref];
					if (c->n_mat > 0 && m >= c->n_mat)
						return fail(GCMX_ERR_INVALID_ARG, "material id out of range");
					inner[(size_t)i] = m;
					mx = std::max(mx, (int)m);
				}
		if (!c->mat_d) HIP_TRY(hipMalloc(&c->mat_d, inner.size()));
		HIP_TRY(hipMemcpy(c->mat_d, inner.data(), inner.size(), hipMemcpyHostToDevice));
		c->max_mat_id = mx;
	}
	refresh_fast(c);
	return GCMX_OK;
}

// Host AoS (reference order, all nodes) <-> device SoA layer.
static void aos_to_soa(const gcmx_ctx* c, const double* aos, double* soa) {
	const Geo& g = c->geo;
	const int D = c->D, M = c->M;
	const long long n0 = c->all_shape[0], n1 = c->all_shape[1], n2 = c->all_shape[2];
	const long long first = g.origin - c->bs * (g.stride[0] + (D > 1 ? g.stride[1] : 0) +
	                                            (D > 2 ? g.stride[2] : 0));
	auto work = [&](long long a0, long long a1) {
		for (long long i0 = a0; i0 < a1; i0++)
			for (long long i1 = 0; i1 < n1; i1++)
				for (long long i2 = 0; i2 < n2; i2++) {
					const long long ref = (i0 * n1 + i1) * n2 + i2;
					const long long dev = first + i0 * g.stride[0] + (D > 1 ? i1 * g.stride[1] : 0) +
					                      (D > 2 ? i2 * g.stride[2] : 0);
					for (int m = 0; m < M; m++) soa[m * g.cs + dev] = aos[ref * M + m];
				}
	};
	const int nt = (int)std::min<long long>(16, std::max<long long>(1, n0 / 8));
	std::vector<std::thread> th;
	for (int t = 0; t < nt; t++) th.emplace_back(work, n0 * t / nt, n0 * (t + 1) / nt);
	for (auto& t : th) t.join();
}

static void soa_to_aos(const gcmx_ctx* c, const double* soa, double* aos) {
	const Geo& g = c->geo;
	const int D = c->D, M = c->M;
	const long long n0 = c->all_shape[0], n1 = c->all_shape[1], n2 = c->all_shape[2];
	const long long first = g.origin - c->bs * (g.stride[0] + (D > 1 ? g.stride[1] : 0) +
	                                            (D > 2 ? g.stride[2] : 0));
	auto work = [&](long long a0, long long a1) {
		for (long long i0 = a0; i0 < a1; i0++)
			for (long long i1 = 0; i1 < n1; i1++)
				for (long long i2 = 0; i2 < n2; i2++) {
					const long long ref = (i0 * n1 + i1) * n2 + i2;
					const long long dev = first + i0 * g.stride[0] + (D > 1 ? i1 * g.stride[1] : 0) +
					                      (D > 2 ? i2 * g.stride[2] : 0);
					for (int m = 0; m < M; m++) aos[ref * M + m] = soa[m * g.cs + dev];
				}
	};
	const int nt = (int)std::min<long long>(16, std::max<long long>(1, n0 / 8));
	std::vector<std::thread> th;
	for (int t = 0; t < nt; t++) th.emplace_back(work, n0 * t / nt, n0 * (t + 1) / nt);
	for (auto& t : th) t.join();
}

gcmx_status gcmx_upload(gcmx_ctx* c, const double* aos) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	s = halo_wait(c);
	if (s) return s;
	if (!aos) return fail(GCMX_ERR_INVALID_ARG, "null host array");
	std::vector<double> soa(c->layer_elems, 0.0);
	aos_to_soa(c, aos, soa.data());
	// Ghost values that are not zero make the two time layers differ in their
	// ghosts, which the fused step (it leaves the state in the other layer)
	// must not assume away: fall back to the per-stage path.
	{
		const Geo& g = c->geo;
		const long long n0 = c->all_shape[0], n1 = c->all_shape[1], n2 = c->all_shape[2];
		bool nz = false;
		for (long long i0 = 0; i0 < n0 && !nz; i0++)
			for (long long i1 = 0; i1 < n1 && !nz; i1++)
				for (long long i2 = 0; i2 < n2 && !nz; i2++) {
					const bool ghost = (i0 < c->bs || i0 >= n0 - c->bs) ||
					                   (c->D > 1 && (i1 < c->bs || i1 >= n1 - c->bs)) ||
					                   (c->D > 2 && (i2 < c->bs || i2 >= n2 - c->bs));
					if (!ghost) continue;
					const long long ref = (i0 * n1 + i1) * n2 + i2;
					for (int m = 0; m < c->M; m++) nz |= aos[ref * c->M + m] != 0.0;
				}
		(void)g;
		if (nz) c->ghosts_touched = true;
	}
	if ((s = wait_stream(c, c->stream, "gcmx_upload")) != GCMX_OK) return s;
	HIP_TRY(hipMemcpy(c->cur, soa.data(), c->layer_elems * sizeof(double), hipMemcpyHostToDevice));
	touch_layer(c);
	return GCMX_OK;
}

gcmx_status gcmx_download(gcmx_ctx* c, double* aos) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	s = halo_wait(c);
	if (s) return s;
	if (!aos) return fail(GCMX_ERR_INVALID_ARG, "null host array");
	std::vector<double> soa(c->layer_elems);
	if ((s = wait_stream(c, c->stream, "gcmx_download")) != GCMX_OK) return s;
	HIP_TRY(hipMemcpy(soa.data(), c->cur, c->layer_elems * sizeof(double), hipMemcpyDeviceToHost));
	soa_to_aos(c, soa.data(), aos);
	return GCMX_OK;
}

gcmx_status gcmx_fill_random(gcmx_ctx* c, const int gs[3], uint64_t seed) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	s = halo_wait(c);
	if (s) return s;
	if (!gs) return fail(GCMX_ERR_INVALID_ARG, "null sizes");
	const int D = c->D;
	int st[3] = {0, 0, 0};
	for (int i = 0; i < D; i++) {
		st[i] = c->desc.start[i];
		if (st[i] < 0 || st[i] + c->desc.sizes[i] > gs[i])
			return fail(GCMX_ERR_INVALID_ARG, "local box outside the global box");
	}
	launch_fill_random(c->cur, c->geo, st, D > 1 ? gs[1] : 1, D > 2 ? gs[2] : 1, seed, c->stream);
	HIP_TRY(hipGetLastError());
	touch_layer(c);
	return GCMX_OK;
}

gcmx_status gcmx_stage(gcmx_ctx* c, int axis, double tau) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (axis < 0 || axis >= c->D) return fail(GCMX_ERR_INVALID_ARG, "axis out of range");
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	return stage_impl(c, axis, tau);
}

// Joins the side streams of the X-slab schedule back into the context stream
// on every exit from gcmx_step, error returns included: later calls (download,
// upload, the next step) are ordered on c->stream only.
struct SlabJoin {
	gcmx_ctx* c;
	bool inner = false, bnd = false;
	~SlabJoin() {
		if (bnd) join(c->ev_bnd, c->bnd_stream);
		if (inner) join(c->ev_join, c->inner_stream);
	}
	// event join; should the event calls fail, a host join keeps the order
	void join(hipEvent_t ev, hipStream_t side) {
		if (hipEventRecord(ev, side) != hipSuccess || hipStreamWaitEvent(c->stream, ev, 0) != hipSuccess)
			(void)hipStreamSynchronize(side);
	}
};

// One 2-D step in one pass (k_step2d, cur -> nxt, then swap): the caller
// checked step2d_admissible.
gcmx_status step2d(gcmx_ctx* c, const Face2* faces = nullptr) {
	const Geo& g = c->geo;
	Timed t(c, "step2d", node_stage_bytes(c) * (double)g.n_inner, c->stream);
	if (!launch_step2d(c->cur, c->nxt, g, c->tabs_d, c->iso2_fast ? c->iso : nullptr, c->stream, &t.kname, faces))
		return fail(GCMX_ERR_UNSUPPORTED, "no 2-D step variant for this configuration");
	HIP_TRY(hipGetLastError());
	std::swap(c->cur, c->nxt);
	touch_layer(c);
	c->last_path = GCMX_PATH_FUSED;
	return GCMX_OK;
}

// One fused step (k_step_tx2 / k_fused_xyz): the caller checked the path.
// `fb`: y/z face conditions (x faces already filled in memory), or null.
// `final`: the step's result is the new state (no separate ODE pass follows).
// Only then may the boundary-first / X-slab schedules post the exchange of the
// new boundary planes inside the step (step_posted); otherwise end_step posts
// the finished layer.  Every step API call thus ends with exactly one post of
// the new state, whatever the rank decided locally (ODE folded or not, one-pass
// or per-stage path, schedule), so the neighbours' posts pair up step by step
// and at the final gcmx_sync (a rank posting a second generation
// after a non-folded ODE mismatched RCCL's send/recv counts; a rank posting one
// step later than its neighbour left the last wait unmatched).
gcmx_status fused_step(gcmx_ctx* c, const FaceBC* fb, bool final) {
	gcmx_status s = GCMX_OK;
	// One pass per step (k_fused_xyz: cur -> nxt, then swap).  Ghost planes of
	// `cur` must hold E_n; with the X-slab schedule the exchange of the NEW
	// boundary planes (E_{n+1}, into the ghost planes of `nxt`) runs while the
	// interior planes are computed.
	const Geo& g = c->geo;
	const int X = g.sizes[0], bs = c->bs;
	const double plane_bytes = node_stage_bytes(c) * (double)g.sizes[1] * g.sizes[2];
	const bool halo = has_halo(c);
	auto xyz = [&](const char* name, int x0, int x1, hipStream_t st, int rows, int xb0 = 0, int xb1 = 0) {
		Timed t(c, name, plane_bytes * ((x1 - x0) + (xb1 - xb0)), st);
		const HetMaterials het{c->het_d, c->mat_d};
		auto launch = c->fp_mode == GCMX_FP_EXACT ? xyz_exact::launch_fused_xyz : xyz_fma::launch_fused_xyz;
		return launch(c->cur, c->nxt, g, c->iso, x0, x1, st, rows, fb, &t.kname, c->iso_het ? &het : nullptr,
		              xb0, xb1);
	};
	const gcmx_schedule sched =
	    c->sched == GCMX_SCHED_AUTO ? (halo ? GCMX_SCHED_BFIRST : GCMX_SCHED_SINGLE) : c->sched;
	bool ok = true;
	// boundary rows per block: 16 beside the interior (XSLAB), 4 alone on the
	// GPU (BFIRST: 2 x 128 blocks for a 512^2 face); GCMX_BOUNDARY_ROWS
	// overrides both (tuning only)
	static const int brows_env = [] {
		const char* e = std::getenv("GCMX_BOUNDARY_ROWS");
		return e ? std::atoi(e) : 0;
	}();
	if (sched == GCMX_SCHED_BFIRST && X >= 4 * bs) {
		// Boundary-first schedule, one stream: the 2 x bs boundary planes (both
		// sides in ONE launch of thin blocks) wait for the halo and run alone on
		// the GPU, the exchange of their NEW planes is posted at once, and the
		// interior planes [bs, X-bs) follow, covering the exchange.  Interior
		// blocks are never resident when the boundary blocks are dispatched, and
		// no cross-stream wait sits on the compute path, so nothing delays the
		// critical path boundary -> exchange -> next step's boundary.
		if (halo) {
			s = halo_ensure(c);
			if (s) return s;
		}
		const int brows = brows_env > 0 ? brows_env : 4;
		ok = xyz("fused_xyz_boundary", 0, bs, c->stream, brows, X - bs, X);
		if (ok && halo && final) {
			std::swap(c->cur, c->nxt);  // E_{n+1}: exchange the new boundary planes
			s = halo_post(c);
			std::swap(c->cur, c->nxt);
			if (s) return s;
			c->step_posted = true;
		}
		ok = ok && xyz("fused_xyz", bs, X - bs, c->stream, c->rows_per_block);
	} else if (sched == GCMX_SCHED_XSLAB && X >= 4 * bs) {
		// X-slab schedule.  The interior planes [bs, X-bs) read no ghost plane:
		// they start at once on the low-priority inner stream, ordered only
		// after the previous step (ev_fork), not after the halo.  The boundary
		// planes wait for the halo and run side by side on the high-priority
		// main and boundary streams in thin 16-row blocks (they finish early, so
		// the exchange of the NEW boundary planes overlaps the interior); then
		// the main stream joins both.  Buffers: the interior writes nxt's inner
		// planes only, the halo writes nxt's ghost planes (no overlap); both read cur.
		SlabJoin join{c};
		HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
		HIP_TRY(hipStreamWaitEvent(c->inner_stream, c->ev_fork, 0));
		join.inner = true;
		ok = xyz("fused_xyz", bs, X - bs, c->inner_stream, c->rows_per_block);
		if (ok && halo && !c->halo_pending && !c->halo_fresh) {
			s = halo_post(c);
			if (s) return s;
		}
		s = halo_wait(c);
		if (s) return s;
		HIP_TRY(hipEventRecord(c->ev_bnd, c->stream));
		HIP_TRY(hipStreamWaitEvent(c->bnd_stream, c->ev_bnd, 0));
		join.bnd = true;
		const int brows = brows_env > 0 ? brows_env : 16;
		ok = ok && xyz("fused_xyz_boundary", 0, bs, c->stream, brows) &&
		     xyz("fused_xyz_boundary", X - bs, X, c->bnd_stream, brows);
		HIP_TRY(hipEventRecord(c->ev_bnd, c->bnd_stream));
		HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_bnd, 0));
		join.bnd = false;
		if (ok && halo && final) {
			std::swap(c->cur, c->nxt);  // E_{n+1} exchanges the new layer
			s = halo_post(c);
			std::swap(c->cur, c->nxt);
			if (s) return s;
			c->step_posted = true;
		}
	} else {
		if (halo) {
			s = halo_ensure(c);
			if (s) return s;
		}
		ok = xyz("fused_xyz", 0, X, c->stream, c->rows_per_block);
		// A slab too thin for the boundary / interior split (X < 4 bs) under the
		// boundary-first or X-slab schedule still keeps their exchange protocol
		// -- its new planes posted right after the step, one post per step --
		// so that it pairs with neighbours that run the split (a group of 8-,
		// 6- and 10-plane slabs otherwise waited forever for a post the thin
		// slab never made).
		if (ok && halo && final && (sched == GCMX_SCHED_BFIRST || sched == GCMX_SCHED_XSLAB)) {
			std::swap(c->cur, c->nxt);
			s = halo_post(c);
			std::swap(c->cur, c->nxt);
			if (s) return s;
			c->step_posted = true;
		}
	}
	if (!ok) return fail(GCMX_ERR_UNSUPPORTED, "fused path launch failed");
	HIP_TRY(hipGetLastError());
	std::swap(c->cur, c->nxt);
	touch_layer(c);
	c->last_path = GCMX_PATH_FUSED;
	return GCMX_OK;
}

}  // extern "C"

namespace {

// The Maxwell ODE a step may carry (gcmx_step_ode): one factor per material.
struct StepOde {
	bool on = false;
	std::vector<double> f;
};

gcmx_status ode_factors(gcmx_ctx* c, double tau, const double* tau0, int n_mat, StepOde& ode) {
	if (c->n_mat == 0) return fail(GCMX_ERR_STATE, "materials not set");
	if (!tau0 || n_mat != c->n_mat) return fail(GCMX_ERR_INVALID_ARG, "one tau0 per material expected");
	ode.on = true;
	ode.f.resize(n_mat);
	for (int m = 0; m < n_mat; m++) ode.f[m] = std::exp(-tau / tau0[m]);  // Ode.hpp:34-35
	return GCMX_OK;
}

gcmx_status ode_apply(gcmx_ctx* c, const std::vector<double>& f);
gcmx_status ode_upload(gcmx_ctx* c, const std::vector<double>& f);

// The ODE rides in the one-pass step's store epilogue when the step runs
// k_step_tx2: over one material (the factor is one number), or over per-node
// materials on the heterogeneous one-pass step (per-material factors, each
// node's own read from LDS).  Call after build_tables (het_ok is per tau).
bool ode_foldable(const gcmx_ctx* c, const StepOde& ode) {
	// rows longer than 512: only the z split has the store epilogue (uniform medium)
	if (!ode.on || c->bs > 2 || (c->geo.sizes[2] > 512 && !(!c->mat_d && zs_admissible(c->geo, c->iso))))
		return false;
	if (!c->mat_d) return ode.f.size() == 1;
	return c->iso_het && c->het_ok && (int)ode.f.size() <= kHetMaxMaterials;
}

// Fills fb's ODE fields for a folded ODE (the HET factors uploaded in stream order).
gcmx_status ode_fold(gcmx_ctx* c, const StepOde& ode, FaceBC& fb) {
	fb.ode_on = 1;
	if (!c->mat_d) {
		fb.ode = ode.f[0];
		return GCMX_OK;
	}
	gcmx_status s = ode_upload(c, ode.f);
	if (s) return s;
	fb.ode_f = c->ode_d;
	return GCMX_OK;
}

// Every step API call ends here: the new state's boundary planes are posted
// unless the one-pass schedule posted them inside the step already.
gcmx_status end_step(gcmx_ctx* c) {
	if (!has_halo(c) || c->step_posted) return GCMX_OK;
	gcmx_status s = halo_wait(c);
	if (s) return s;
	return halo_post(c);
}

gcmx_status step_body(gcmx_ctx* c, double tau, const StepOde& ode);

gcmx_status step_impl(gcmx_ctx* c, double tau, const StepOde& ode) {
	c->step_posted = false;
	gcmx_status s = step_body(c, tau, ode);
	return s ? s : end_step(c);
}

gcmx_status step_body(gcmx_ctx* c, double tau, const StepOde& ode) {
	gcmx_status s = build_tables(c, tau);
	if (s) return s;
	c->last_ode_fused = false;
	if (c->D == 2 && effective_path(c) == GCMX_PATH_FUSED) {
		s = step2d(c);
		if (s) return s;
		return ode.on ? ode_apply(c, ode.f) : GCMX_OK;
	}
	if (effective_path(c) != GCMX_PATH_FUSED || c->faces_written != 0 || (c->iso_het && !c->het_ok)) {
		for (int a = 0; a < c->D; a++) {
			s = stage_impl(c, a, tau);
			if (s) return s;
		}
		return ode.on ? ode_apply(c, ode.f) : GCMX_OK;
	}
	if (ode_foldable(c, ode)) {
		FaceBC fb{};
		s = ode_fold(c, ode, fb);
		if (s) return s;
		s = fused_step(c, &fb, true);
		if (s) return s;
		c->last_ode_fused = true;
		return GCMX_OK;
	}
	s = fused_step(c, nullptr, !ode.on);
	if (s) return s;
	return ode.on ? ode_apply(c, ode.f) : GCMX_OK;
}

gcmx_status step_faces_impl(gcmx_ctx* c, double tau, const gcmx_face* faces, const StepOde& ode);

}  // namespace

extern "C" {

gcmx_status gcmx_step(gcmx_ctx* c, double tau) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	return step_impl(c, tau, StepOde{});
}

gcmx_status gcmx_step_faces(gcmx_ctx* c, double tau, const gcmx_face* faces) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	if (!faces) return fail(GCMX_ERR_INVALID_ARG, "null faces");
	return step_faces_impl(c, tau, faces, StepOde{});
}

gcmx_status gcmx_step_ode(gcmx_ctx* c, double tau, const gcmx_face* faces, const double* tau0, int n_mat) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	StepOde ode;
	if ((s = ode_factors(c, tau, tau0, n_mat, ode)) != GCMX_OK) return s;
	return faces ? step_faces_impl(c, tau, faces, ode) : step_impl(c, tau, ode);
}

int gcmx_last_ode_fused(gcmx_ctx* c) { return c && c->last_ode_fused ? 1 : 0; }

}  // extern "C"

namespace {

gcmx_status step_faces_body(gcmx_ctx* c, double tau, const gcmx_face* faces, const StepOde& ode);

gcmx_status step_faces_impl(gcmx_ctx* c, double tau, const gcmx_face* faces, const StepOde& ode) {
	c->step_posted = false;
	gcmx_status s = step_faces_body(c, tau, faces, ode);
	return s ? s : end_step(c);
}

gcmx_status step_faces_body(gcmx_ctx* c, double tau, const gcmx_face* faces, const StepOde& ode) {
	gcmx_status s = GCMX_OK;
	c->last_ode_fused = false;
	const int D = c->D;
	BorderQ bq[6] = {};
	unsigned on = 0;
	for (int f = 0; f < 2 * D; f++) {
		if (!faces[f].enabled) continue;
		s = border_q(c, faces[f].n_quantities, faces[f].quantities, faces[f].values, bq[f]);
		if (s) return s;
		on |= 1u << f;
	}
	s = build_tables(c, tau);
	if (s) return s;
	auto fill = [&](int f) -> gcmx_status {
		s = halo_wait(c);
		if (s) return s;
		Timed t(c, "face_fill", 0.0, c->stream);
		launch_face_fill(c->cur, c->geo, f / 2, (f & 1) ? 1 : -1, bq[f], c->stream);
		HIP_TRY(hipGetLastError());
		c->faces_written |= 1u << f;
		return GCMX_OK;
	};
	if (D == 2 && step2d_faces_admissible(c, on)) {
		// One 2-D pass: x faces in memory, y faces formed in the pass (Face2); a
		// y face with PRESSURE (its trace needs components the pass does not form
		// at ghosts) keeps the per-stage path.
		Face2 f2{};
		bool ok = true;
		for (int f = 2; f < 4 && ok; f++) {
			if (!((on >> f) & 1u)) continue;
			f2.on |= 1u << (f - 2);
			for (int k = 0; k < bq[f].n; k++) {
				const int comp = quantity_comp(D, bq[f].q[k]);
				if (comp < 0) {
					ok = false;
					break;
				}
				f2.mask[f - 2] |= 1u << comp;
				f2.two_v[f - 2][comp] = 2 * bq[f].v[k];  // the last setting of a component wins
			}
		}
		if (ok) {
			for (int f = 0; f < 2; f++)
				if ((on >> f) & 1u) {
					s = fill(f);
					if (s) return s;
				}
			s = step2d(c, &f2);
			if (s) return s;
			return ode.on ? ode_apply(c, ode.f) : GCMX_OK;
		}
	}
	// One pass: x faces in memory, y/z faces as FaceBC; the y/z faces must be
	// free of PRESSURE (its trace needs components the fused ghosts do not form)
	// and no face may hold ghosts written earlier but not refreshed now.
	bool fused = D == 3 && effective_path(c) == GCMX_PATH_FUSED && fused_faces_supported(c->geo) &&
	             (c->geo.sizes[2] <= 512 || (!c->mat_d && zs_admissible(c->geo, c->iso))) &&
	             (c->faces_written & ~on) == 0 && (!c->iso_het || c->het_ok);
	FaceBC fb{};
	for (int f = 2; f < 6 && fused; f++) {
		if (!((on >> f) & 1u)) continue;
		fb.on |= 1u << (f - 2);
		for (int k = 0; k < bq[f].n; k++) {
			const int comp = quantity_comp(D, bq[f].q[k]);
			if (comp < 0) {
				fused = false;  // PRESSURE
				break;
			}
			fb.mask[f - 2] |= 1u << comp;
			fb.two_v[f - 2][comp] = 2 * bq[f].v[k];  // the last setting of a component wins
		}
	}
	if (fused) {
		for (int f = 0; f < 2; f++)
			if ((on >> f) & 1u) {
				s = fill(f);
				if (s) return s;
			}
		const bool fold = ode_foldable(c, ode);
		if (fold) {
			s = ode_fold(c, ode, fb);
			if (s) return s;
		}
		s = fused_step(c, (fb.on || fold) ? &fb : nullptr, !(ode.on && !fold));
		if (s) return s;
		c->last_ode_fused = fold;
		return (ode.on && !fold) ? ode_apply(c, ode.f) : GCMX_OK;
	}
	for (int a = 0; a < D; a++) {
		for (int f = 2 * a; f < 2 * a + 2; f++)
			if ((on >> f) & 1u) {
				s = fill(f);
				if (s) return s;
			}
		s = stage_impl(c, a, tau);
		if (s) return s;
	}
	return ode.on ? ode_apply(c, ode.f) : GCMX_OK;
}

}  // namespace

extern "C" {

gcmx_status gcmx_face_map_create(gcmx_ctx* c, const uint8_t* const node_condition[6], gcmx_face_map** out) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!out || !node_condition) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	*out = nullptr;
	auto m = std::unique_ptr<gcmx_face_map, void (*)(gcmx_face_map*)>(new gcmx_face_map(), gcmx_face_map_destroy);
	m->ctx = c;
	for (int f = 0; f < 2 * c->D; f++) {
		if (!node_condition[f]) continue;
		size_t n = 1;
		for (int d = 0; d < c->D; d++)
			if (d != f / 2) n *= (size_t)c->geo.sizes[d];
		unsigned used = 0;
		for (size_t i = 0; i < n; i++) {
			const unsigned v = node_condition[f][i];
			if (v == kNoFaceCond) continue;
			if (v >= (unsigned)kMaxFaceConds)
				return fail(GCMX_ERR_INVALID_ARG, "face map: condition index >= " + std::to_string(kMaxFaceConds));
			used |= 1u << v;
		}
		if (!used) continue;  // no condition on this face: its ghosts stay as they are
		m->used[f] = used;
		bool whole = true;  // one condition on every node: the face is uniform, no map needed
		for (size_t i = 0; i < n && whole; i++) whole = node_condition[f][i] == node_condition[f][0];
		if (whole) {
			m->uni[f] = node_condition[f][0];
			continue;
		}
		HIP_TRY(hipMalloc(&m->map_d[f], n));
		HIP_TRY(hipMemcpy(m->map_d[f], node_condition[f], n, hipMemcpyHostToDevice));
	}
	HIP_TRY(hipMalloc(&m->bq_d, kMaxFaceConds * sizeof(BorderQ)));
	HIP_TRY(hipMalloc(&m->fc_d, kMaxFaceConds * sizeof(FaceCond)));
	*out = m.release();
	return GCMX_OK;
}

void gcmx_face_map_destroy(gcmx_face_map* m) {
	if (!m) return;
	if (m->ctx) {
		(void)hipSetDevice(m->ctx->device);
		(void)hipStreamSynchronize(m->ctx->stream);  // a pending step may still read the maps
	}
	for (uint8_t* p : m->map_d) (void)hipFree(p);
	(void)hipFree(m->bq_d);
	(void)hipFree(m->fc_d);
	delete m;
}

static gcmx_status step_face_map_body(gcmx_ctx* c, double tau, const gcmx_face_map* m, int n_cond,
                                      const gcmx_face* conds);

gcmx_status gcmx_step_face_map(gcmx_ctx* c, double tau, const gcmx_face_map* m, int n_cond,
                               const gcmx_face* conds) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	c->step_posted = false;
	s = step_face_map_body(c, tau, m, n_cond, conds);
	return s ? s : end_step(c);
}

static gcmx_status step_face_map_body(gcmx_ctx* c, double tau, const gcmx_face_map* m, int n_cond,
                                      const gcmx_face* conds) {
	gcmx_status s = GCMX_OK;
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	if (!m || m->ctx != c) return fail(GCMX_ERR_INVALID_ARG, "face map of another context");
	if (n_cond < 0 || n_cond > kMaxFaceConds || (n_cond > 0 && !conds))
		return fail(GCMX_ERR_INVALID_ARG, "0.." + std::to_string(kMaxFaceConds) + " conditions expected");
	const int D = c->D;
	unsigned on = 0;
	for (int f = 0; f < 2 * D; f++)
		if (m->map_d[f] || m->uni[f] >= 0) {
			if (m->used[f] >> n_cond) return fail(GCMX_ERR_INVALID_ARG, "the face map names a condition not given");
			on |= 1u << f;
		}
	FaceTables t{};
	t.n = n_cond;
	unsigned pressure = 0;  // conditions that set PRESSURE (the fused ghosts cannot form its trace)
	for (int k = 0; k < n_cond; k++) {
		if ((s = border_q(c, conds[k].n_quantities, conds[k].quantities, conds[k].values, t.bq[k])) != GCMX_OK)
			return s;
		FaceCond& fc = t.fc[k];
		for (int q = 0; q < t.bq[k].n; q++) {
			const int comp = quantity_comp(D, t.bq[k].q[q]);
			if (comp < 0) {
				pressure |= 1u << k;
				continue;
			}
			fc.mask |= 1u << comp;
			fc.two_v[comp] = 2 * t.bq[k].v[q];  // the last setting of a component wins
		}
	}
	if ((s = build_tables(c, tau)) != GCMX_OK) return s;
	if ((s = halo_wait(c)) != GCMX_OK) return s;
	launch_set_face_tables(m->bq_d, m->fc_d, t, c->stream);
	HIP_TRY(hipGetLastError());
	c->last_ode_fused = false;
	bool fused = D == 3 && effective_path(c) == GCMX_PATH_FUSED && fused_faces_supported(c->geo) &&
	             (c->geo.sizes[2] <= 512 || (!c->mat_d && zs_admissible(c->geo, c->iso))) &&
	             (c->faces_written & ~on) == 0 && (!c->iso_het || c->het_ok);
	for (int f = 2; f < 2 * D && fused; f++)
		if (m->used[f] & pressure) fused = false;
	auto fill = [&](int f) -> gcmx_status {
		gcmx_status st = halo_wait(c);
		if (st) return st;
		Timed tm(c, "face_fill", 0.0, c->stream);
		if (m->map_d[f])
			launch_face_fill_map(c->cur, c->geo, f / 2, (f & 1) ? 1 : -1, m->map_d[f], m->bq_d, c->stream);
		else
			launch_face_fill(c->cur, c->geo, f / 2, (f & 1) ? 1 : -1, t.bq[m->uni[f]], c->stream);
		HIP_TRY(hipGetLastError());
		c->faces_written |= 1u << f;
		return GCMX_OK;
	};
	if (fused) {
		// x faces in memory, y/z faces formed inside the one-pass step per face node
		for (int f = 0; f < 2; f++)
			if (((on >> f) & 1u) && (s = fill(f)) != GCMX_OK) return s;
		FaceBC fb{};
		for (int f = 2; f < 6; f++)
			if (m->map_d[f]) {
				fb.on |= 1u << (f - 2);
				fb.map[f - 2] = m->map_d[f];
			} else if (m->uni[f] >= 0) {  // uniform face: the condition as kernel arguments
				const FaceCond& fc = t.fc[m->uni[f]];
				fb.on |= 1u << (f - 2);
				fb.mask[f - 2] = fc.mask;
				for (int j = 0; j < 9; j++) fb.two_v[f - 2][j] = fc.two_v[j];
			}
		fb.conds = m->fc_d;
		return fused_step(c, fb.on ? &fb : nullptr, true);
	}
	for (int a = 0; a < D; a++) {  // BorderConditions::apply(mesh, a), then the stage (Engine.cpp:90-121)
		for (int f = 2 * a; f < 2 * a + 2; f++)
			if (((on >> f) & 1u) && (s = fill(f)) != GCMX_OK) return s;
		if ((s = stage_impl(c, a, tau)) != GCMX_OK) return s;
	}
	return GCMX_OK;
}

gcmx_status gcmx_set_fp_mode(gcmx_ctx* c, gcmx_fp_mode mode) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (mode != GCMX_FP_FMA && mode != GCMX_FP_EXACT) return fail(GCMX_ERR_INVALID_ARG, "unknown fp mode");
	c->fp_mode = mode;
	return GCMX_OK;
}

gcmx_status gcmx_get_fp_mode(const gcmx_ctx* c, gcmx_fp_mode* mode) {
	if (!c || !mode) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	*mode = c->fp_mode;
	return GCMX_OK;
}

gcmx_status gcmx_set_step_schedule(gcmx_ctx* c, gcmx_schedule sched, int rows_per_block) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null context");
	if (sched < GCMX_SCHED_AUTO || sched > GCMX_SCHED_BFIRST)
		return fail(GCMX_ERR_INVALID_ARG, "bad schedule");
	if (rows_per_block < 0 || rows_per_block > 4096)
		return fail(GCMX_ERR_INVALID_ARG, "rows_per_block must be 0 (automatic) .. 4096");
	c->sched = sched;
	c->rows_per_block = rows_per_block;
	return GCMX_OK;
}

gcmx_status gcmx_set_kernel_path(gcmx_ctx* c, gcmx_path p) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null context");
	if (p < GCMX_PATH_AUTO || p > GCMX_PATH_FUSED) return fail(GCMX_ERR_INVALID_ARG, "bad path");
	c->path = p;
	return GCMX_OK;
}

gcmx_path gcmx_effective_path(gcmx_ctx* c) { return c ? effective_path(c) : GCMX_PATH_GENERIC; }
gcmx_path gcmx_last_step_path(gcmx_ctx* c) { return c ? c->last_path : GCMX_PATH_AUTO; }

static gcmx_status check_face_nodes(gcmx_ctx* c, int axis, int side, int n_nodes, const int* nodes) {
	if (axis < 0 || axis >= c->D || (side != 1 && side != -1) || n_nodes < 0 || (n_nodes > 0 && !nodes))
		return fail(GCMX_ERR_INVALID_ARG, "bad border-fill arguments");
	const int D = c->D;
	for (int i = 0; i < n_nodes; i++) {
		for (int d = 0; d < D; d++) {
			const int v = nodes[i * D + d];
			if (v < 0 || v >= c->geo.sizes[d]) return fail(GCMX_ERR_INVALID_ARG, "face node out of range");
		}
		const int want = side > 0 ? c->geo.sizes[axis] - 1 : 0;
		if (nodes[i * D + axis] != want) return fail(GCMX_ERR_INVALID_ARG, "node not on the face");
	}
	return GCMX_OK;
}

gcmx_status gcmx_border_fill(gcmx_ctx* c, int axis, int side, int n_nodes, const int* nodes,
                             int n_q, const int* qs, const double* vals) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if ((s = check_face_nodes(c, axis, side, n_nodes, nodes)) != GCMX_OK) return s;
	BorderQ bq;
	if ((s = border_q(c, n_q, qs, vals, bq)) != GCMX_OK) return s;
	c->ghosts_touched = true;
	s = halo_wait(c);
	if (s) return s;
	if (n_nodes == 0) return GCMX_OK;
	const size_t need = (size_t)n_nodes * c->D;
	HIP_TRY(hipStreamSynchronize(c->stream));  // scratch reuse (gcmx_border_apply has none)
	if (need > c->nodes_cap) {
		(void)hipFree(c->nodes_d);
		c->nodes_d = nullptr;
		c->nodes_cap = 0;
		HIP_TRY(hipMalloc(&c->nodes_d, need * sizeof(int)));
		c->nodes_cap = need;
	}
	HIP_TRY(hipMemcpy(c->nodes_d, nodes, need * sizeof(int), hipMemcpyHostToDevice));
	launch_border_fill(c->cur, c->geo, axis, side > 0 ? -1 : 1, n_nodes, c->nodes_d, bq, c->stream);
	HIP_TRY(hipGetLastError());
	return GCMX_OK;
}

gcmx_status gcmx_border_nodes_create(gcmx_ctx* c, int axis, int side, int n_nodes, const int* nodes,
                                     gcmx_border_nodes** out) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!out) return fail(GCMX_ERR_INVALID_ARG, "null output");
	*out = nullptr;
	if ((s = check_face_nodes(c, axis, side, n_nodes, nodes)) != GCMX_OK) return s;
	auto* h = new gcmx_border_nodes();
	h->ctx = c;
	h->axis = axis;
	h->side = side;
	h->n = n_nodes;
	if (n_nodes > 0) {
		const size_t bytes = (size_t)n_nodes * c->D * sizeof(int);
		if (hipMalloc(&h->nodes_d, bytes) != hipSuccess) {
			delete h;
			return fail(GCMX_ERR_OOM, "device allocation failed");
		}
		if (hipMemcpy(h->nodes_d, nodes, bytes, hipMemcpyHostToDevice) != hipSuccess) {
			(void)hipFree(h->nodes_d);
			delete h;
			return fail(GCMX_ERR_HIP, "node list upload failed");
		}
	}
	*out = h;
	return GCMX_OK;
}

gcmx_status gcmx_border_apply(gcmx_ctx* c, const gcmx_border_nodes* h, int n_q, const int* qs,
                              const double* vals) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!h || h->ctx != c) return fail(GCMX_ERR_INVALID_ARG, "node list of another context");
	BorderQ bq;
	if ((s = border_q(c, n_q, qs, vals, bq)) != GCMX_OK) return s;
	c->ghosts_touched = true;
	s = halo_wait(c);
	if (s) return s;
	if (h->n == 0) return GCMX_OK;
	Timed t(c, "border_fill", 0.0, c->stream);
	launch_border_fill(c->cur, c->geo, h->axis, h->side > 0 ? -1 : 1, h->n, h->nodes_d, bq, c->stream);
	HIP_TRY(hipGetLastError());
	return GCMX_OK;
}

void gcmx_border_nodes_destroy(gcmx_border_nodes* h) {
	if (!h) return;
	if (h->ctx) {
		(void)hipSetDevice(h->ctx->device);
		(void)hipStreamSynchronize(h->ctx->stream);  // a pending fill may still read the list
	}
	(void)hipFree(h->nodes_d);
	delete h;
}

gcmx_status gcmx_ode_maxwell(gcmx_ctx* c, double tau, const double* tau0, int n_mat) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!std::isfinite(tau)) return fail(GCMX_ERR_INVALID_ARG, "non-finite time step");
	StepOde ode;
	if ((s = ode_factors(c, tau, tau0, n_mat, ode)) != GCMX_OK) return s;
	return ode_apply(c, ode.f);
}

}  // extern "C"

namespace {

// k_scale_stress over the current layer (the separate ODE pass).
// Per-material factors into the context's device slot: they travel as kernel
// arguments, ordered on the stream after the previous launch that read the
// slot -- no host sync.
gcmx_status ode_upload(gcmx_ctx* c, const std::vector<double>& f) {
	if (!c->ode_d) HIP_TRY(hipMalloc(&c->ode_d, 256 * sizeof(double)));
	OdeFactors v{};
	v.n = (int)f.size();
	for (int m = 0; m < v.n; m++) v.f[m] = f[m];
	launch_set_factors(c->ode_d, v, c->stream);
	HIP_TRY(hipGetLastError());
	return GCMX_OK;
}

gcmx_status ode_apply(gcmx_ctx* c, const std::vector<double>& f) {
	gcmx_status s = halo_wait(c);
	if (s) return s;
	if (!c->mat_d) {
		Timed t(c, "ode_maxwell", 2.0 * 8.0 * (c->M - c->D) * (double)c->geo.n_inner, c->stream);
		launch_scale_stress(c->cur, c->geo, nullptr, nullptr, f[0], c->stream);
	} else {
		gcmx_status s2 = ode_upload(c, f);
		if (s2) return s2;
		Timed t(c, "ode_maxwell", (2.0 * 8.0 * (c->M - c->D) + 1.0) * (double)c->geo.n_inner, c->stream);
		launch_scale_stress(c->cur, c->geo, c->mat_d, c->ode_d, 0.0, c->stream);
	}
	HIP_TRY(hipGetLastError());
	touch_layer(c);
	return GCMX_OK;
}

}  // namespace

extern "C" {

gcmx_status gcmx_copy_box(gcmx_ctx* dst, const int dmin[3], const int dmax[3], gcmx_ctx* src,
                          const int smin[3]) {
	gcmx_status s = check_ctx(dst);
	if (s) return s;
	if (!src || !dmin || !dmax || !smin || src->D != dst->D || src->M != dst->M ||
	    src->device != dst->device)
		return fail(GCMX_ERR_INVALID_ARG, "bad copy-box arguments");
	const int D = dst->D;
	int ext[3] = {1, 1, 1}, dm[3] = {0, 0, 0}, sm[3] = {0, 0, 0};
	for (int d = 0; d < D; d++) {
		ext[d] = dmax[d] - dmin[d];
		dm[d] = dmin[d];
		sm[d] = smin[d];
		if (ext[d] <= 0) return fail(GCMX_ERR_INVALID_ARG, "empty box");
		if (dmin[d] < -dst->bs || dmax[d] > dst->geo.sizes[d] + dst->bs || smin[d] < -src->bs ||
		    smin[d] + ext[d] > src->geo.sizes[d] + src->bs)
			return fail(GCMX_ERR_INVALID_ARG, "box outside the grid");
	}
	// A 3-D box inside the x ghost planes ([-bs, 0) or [X, X + bs): a contact
	// along x, ContactCopier for stage 0) fills exactly what the one-pass step
	// reads as x ghosts, like the X-slab halo, so the fused path stays
	// admissible; any other ghost write selects the per-stage path.
	const bool x_ghosts_only = D == 3 && (dmax[0] <= 0 || dmin[0] >= dst->geo.sizes[0]);
	if (!x_ghosts_only) dst->ghosts_touched = true;
	if ((s = halo_wait(dst)) != GCMX_OK || (s = halo_wait(src)) != GCMX_OK) return s;
	// order the copy after the source's pending work
	HIP_TRY(hipEventRecord(src->ev_ready, src->stream));
	HIP_TRY(hipStreamWaitEvent(dst->stream, src->ev_ready, 0));
	launch_copy_box(dst->cur, dst->geo, src->cur, src->geo, dm, sm, ext, dst->stream);
	HIP_TRY(hipGetLastError());
	touch_layer(dst);
	HIP_TRY(hipEventRecord(dst->ev_ready, dst->stream));
	HIP_TRY(hipStreamWaitEvent(src->stream, dst->ev_ready, 0));
	return GCMX_OK;
}

gcmx_status gcmx_comm_unique_id(uint8_t id[GCMX_UNIQUE_ID_BYTES]) {
	static_assert(sizeof(ncclUniqueId) <= GCMX_UNIQUE_ID_BYTES, "unique id size");
	if (!id) return fail(GCMX_ERR_INVALID_ARG, "null id");
	ncclUniqueId u;
	if (ncclGetUniqueId(&u) != ncclSuccess) return fail(GCMX_ERR_COMM, "ncclGetUniqueId failed");
	std::memset(id, 0, GCMX_UNIQUE_ID_BYTES);
	std::memcpy(id, &u, sizeof(u));
	return GCMX_OK;
}

// Channels per peer the automatic rule picks for an X slab of `X` planes on a
// grid of Y x Z rows (see gcmx_comm_init_opts).  With RCCL's default, one
// step's exchange group (a send and a receive per halo component and
// neighbour) runs as SIX kernel launches: the first beside the interior, the
// other five after it, on the next step's critical path.  An explicit
// NCCL_NCHANNELS_PER_PEER makes it ONE launch, whose CTAs must find CUs the
// interior leaves free (an interior block holds a whole CU), else they crawl
// until interior blocks retire.  The one-rank self-exchange on MI355X
//  ran 2 CTAs per channel: 64-plane slabs (16 CUs free) 0.70 ->
// 0.62-0.65 ms/step with 4-8 channels, 128-plane slabs (8 free) 1.17 -> 1.10
// with 2-4 (1.28-1.30 with 6-8), 256-plane slabs (4 free) best with RCCL's
// default.  A rank with two distinct peers may need up to twice the CTAs, so
// the count is sized for that: free CUs / 4, i.e. 4 with >= 16 free CUs, 2 with
// >= 8, else RCCL's own (0).
static int channels_for_slab(int X, int Y, int Z, int bs, int rows_per_block, int cus) {
	// the one-pass step's launch geometry of an X x Y x Z slab (only what
	// step_free_cus reads: sizes, bs, the layout's 32-bit addressing bound)
	Geo g{};
	g.D = 3;
	g.M = 9;
	g.bs = bs;
	g.sizes[0] = X;
	g.sizes[1] = Y;
	g.sizes[2] = Z;
	const long long row = round_up(round_up(bs, kRowAlign) + Z + bs, kRowAlign);
	g.stride[2] = 1;
	g.stride[1] = row;
	g.stride[0] = row * (Y + 2LL * bs);
	g.cs = round_up(g.stride[0] * (X + 2LL * bs), 64);
	const int free_cus = X > 2 * bs ? step_free_cus(g, bs, X - bs, rows_per_block, cus) : -1;
	return free_cus >= 16 ? 4 : free_cus >= 8 ? 2 : 0;
}

// Process-wide: RCCL reads NCCL_NCHANNELS_PER_PEER once per process, so the
// channels per peer of every communicator in the process are those in effect
// when its first one was created (g_rccl_channels, -1 before that);
// g_rccl_user_env: the user set NCCL_NCHANNELS_PER_PEER, which overrides the rule.
static std::mutex g_rccl_mu;
static int g_rccl_channels = -1;
static bool g_rccl_user_env = false;

static int env_int(const char* name, int dflt) {
	const char* e = std::getenv(name);
	return (e && *e) ? std::atoi(e) : dflt;
}

gcmx_status gcmx_comm_init_opts(gcmx_ctx* c, const uint8_t id[GCMX_UNIQUE_ID_BYTES], int nranks, int rank,
                                int left, int right, const gcmx_comm_options* opt) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	// A neighbour equal to this rank is accepted only in a one-rank communicator
	// (the self-exchange that runs the RCCL transport on a one-GPU box, gcmx.h).
	if (!id || nranks < 1 || rank < 0 || rank >= nranks || left >= nranks || right >= nranks ||
	    (nranks > 1 && (left == rank || right == rank)))
		return fail(GCMX_ERR_INVALID_ARG, "bad communicator arguments");
	if (c->comm || c->lc || c->comm_dead) return fail(GCMX_ERR_STATE, "communicator already initialised");
	gcmx_comm_options o;
	if (opt) {
		o = *opt;
	} else {  // defaults, each overridable from the environment (gcmx.h)
		o.global_x = 0;
		o.channels_per_peer = env_int("GCMX_COMM_CHANNELS_PER_PEER", -1);
		o.min_ctas = env_int("GCMX_COMM_MIN_CTAS", -1);
		o.max_ctas = env_int("GCMX_COMM_MAX_CTAS", -1);
		o.timeout_s = 0;
	}
	if (o.global_x < 0 || o.channels_per_peer < -1 || o.channels_per_peer > 64)
		return fail(GCMX_ERR_INVALID_ARG, "bad communicator options");
	ncclUniqueId u;
	std::memcpy(&u, id, sizeof(u));
	// The exchange runs beside the interior kernel, which saturates HBM: a
	// transfer with few blocks in flight is starved and stops hiding behind it
	// (loopback measurement), so ask RCCL for at least 16 blocks
	// (min_ctas; 0 leaves RCCL's own choice), at most 32 (RCCL rejects a minimum
	// without a maximum).
	const int min_ctas = o.min_ctas >= 0 ? o.min_ctas : 16;
	const int max_ctas = o.max_ctas >= 0 ? o.max_ctas : 32;
	// Channels per peer: both ends of a p2p connection must use the same count,
	// so the automatic rule uses only inputs every rank holds alike -- the global
	// X extent, the rank count, Y, Z, borderSize and the library's block rule --
	// applied to the THINNEST slab of an even split (floor(global_x / nranks)
	// planes); a one-rank communicator (the self-exchange) uses its own slab.
	// Without global_x the rule cannot be rank-consistent: RCCL's default
	// (gcmx_comm_channels_rule).  The value reaches RCCL through
	// NCCL_NCHANNELS_PER_PEER, which RCCL reads ONCE per process: the checked
	// contract below sets it (only) before the process's first communicator and
	// refuses a later communicator that needs another count (GCMX_ERR_STATE)
	// instead of letting it silently run with the first one's.
	const int Dg = c->geo.D;
	const int want = o.channels_per_peer >= 0
	                     ? o.channels_per_peer
	                     : gcmx_comm_channels_rule(o.global_x, nranks, c->geo.sizes[0], Dg > 1 ? c->geo.sizes[1] : 1,
	                                               Dg > 2 ? c->geo.sizes[2] : 1, c->bs, c->rows_per_block, 0);
	{
		std::lock_guard<std::mutex> lk(g_rccl_mu);
		if (g_rccl_channels < 0) {  // the process's first communicator: RCCL's value is still open
			if (const char* e = std::getenv("NCCL_NCHANNELS_PER_PEER")) {
				g_rccl_user_env = true;  // the user's choice overrides the rule
				g_rccl_channels = std::atoi(e);
			} else {
				if (want > 0) setenv("NCCL_NCHANNELS_PER_PEER", std::to_string(want).c_str(), 1);
				g_rccl_channels = want;
			}
		} else if (!g_rccl_user_env && want != g_rccl_channels) {
			return fail(GCMX_ERR_STATE,
			            "RCCL channels per peer are fixed at " + std::to_string(g_rccl_channels) +
			                " in this process (RCCL reads NCCL_NCHANNELS_PER_PEER once, at its first communicator); "
			                "this communicator needs " +
			                std::to_string(want) +
			                ": pass gcmx_comm_options.channels_per_peer = " + std::to_string(g_rccl_channels) +
			                " (every rank alike), or create it in a process of its own");
		}
		c->channels_per_peer = g_rccl_channels;
	}
	c->comm_timeout_s = o.timeout_s > 0 ? o.timeout_s : comm_timeout_seconds();
	// Non-blocking communicator: every RCCL call returns at once and its state is
	// polled (comm_settle) under the timeout, so a dead or missing peer surfaces
	// as GCMX_ERR_COMM (after ncclCommAbort) instead of a hang.
	ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
	cfg.blocking = 0;
	if (min_ctas > 0) {
		cfg.minCTAs = min_ctas;
		cfg.maxCTAs = max_ctas > min_ctas ? max_ctas : min_ctas;
	}
	ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, u, rank, &cfg);
	if (r != ncclSuccess && r != ncclInProgress) {
		if (c->comm) (void)ncclCommAbort(c->comm);
		c->comm = nullptr;
		return fail(GCMX_ERR_COMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
	}
	if ((s = comm_settle(c, "ncclCommInitRankConfig")) != GCMX_OK) return s;
	c->nranks = nranks;
	c->rank = rank;
	c->left = left;
	c->right = right;
	return GCMX_OK;
}

gcmx_status gcmx_comm_init(gcmx_ctx* c, const uint8_t id[GCMX_UNIQUE_ID_BYTES], int nranks,
                           int rank, int left, int right) {
	return gcmx_comm_init_opts(c, id, nranks, rank, left, right, nullptr);
}

int gcmx_comm_channels_per_peer(const gcmx_ctx* c) { return c ? c->channels_per_peer : -1; }

int gcmx_comm_channels_rule(int global_x, int nranks, int local_x, int Y, int Z, int bs, int rows_per_block,
                            int cus) {
	if (nranks < 1 || global_x < 0 || local_x < 1 || Y < 1 || Z < 1 || bs < 1 || bs > kMaxBs) return -1;
	if (nranks == 1) return channels_for_slab(local_x, Y, Z, bs, rows_per_block, cus);
	if (global_x == 0) return 0;  // not rank-consistent without the global extent: RCCL's default
	return channels_for_slab(global_x / nranks, Y, Z, bs, rows_per_block, cus);
}

long long gcmx_comm_posted_calls(const gcmx_ctx* c) { return c ? c->halo_posted_calls : -1; }

gcmx_status gcmx_comm_test_stall(gcmx_ctx* c, int on) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null context");
	c->comm_stall = on != 0;
	return GCMX_OK;
}

gcmx_status gcmx_comm_init_loopback(gcmx_ctx* c, double gbps_per_direction, int blocks) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (c->D < 2) return fail(GCMX_ERR_INVALID_ARG, "X-slab halo needs dim >= 2");
	if (!(gbps_per_direction >= 0) || blocks < 1 || blocks > 1024)
		return fail(GCMX_ERR_INVALID_ARG, "loopback: rate >= 0 GB/s and 1..1024 blocks expected");
	if (c->comm || c->lc || c->loop) return fail(GCMX_ERR_STATE, "communicator already initialised");
	if (c->geo.sizes[0] < c->bs) return fail(GCMX_ERR_INVALID_ARG, "loopback: slab thinner than borderSize");
	if (c->geo.stride[0] % 2 != 0 || c->geo.cs % 2 != 0)
		return fail(GCMX_ERR_UNSUPPORTED, "loopback: planes not 16-byte aligned");
	if ((s = halo_wait(c)) != GCMX_OK) return s;
	c->loop = true;
	c->loop_gbps = gbps_per_direction;
	c->loop_blocks = blocks;
	c->nranks = 1;
	c->rank = 0;
	c->left = c->right = 0;  // itself, periodically
	touch_layer(c);
	return GCMX_OK;
}

gcmx_status gcmx_halo_exchange(gcmx_ctx* c) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	return halo_exchange_impl(c);
}

gcmx_status gcmx_halo_exchange_group(gcmx_ctx* const* slabs, int n) {
	if (!slabs || n < 1) return fail(GCMX_ERR_INVALID_ARG, "bad slab list");
	for (int i = 0; i < n; i++) {
		gcmx_ctx* c = slabs[i];
		if (!c || c->D < 2 || c->n_mat <= 0) return fail(GCMX_ERR_INVALID_ARG, "bad slab");
		if (c->lc) return fail(GCMX_ERR_STATE, "slab belongs to an in-process group (gcmx_comm_init_local)");
		if (i > 0) {
			const gcmx_ctx* p = slabs[i - 1];
			bool ok = p->D == c->D && p->bs == c->bs && p->desc.start[0] + p->geo.sizes[0] == c->desc.start[0];
			for (int d = 1; d < c->D; d++) ok = ok && p->geo.sizes[d] == c->geo.sizes[d] && p->desc.start[d] == c->desc.start[d];
			if (!ok) return fail(GCMX_ERR_INVALID_ARG, "slabs are not X-adjacent");
		}
	}
	for (int i = 0; i < n; i++) {
		gcmx_status s = halo_wait(slabs[i]);
		if (s) return s;
	}
	if (n == 1) return GCMX_OK;
	gcmx_ctx* lead = slabs[0];
	// every pair's copies run on the lead's comm stream: the lead's device touches
	// both sides of each pair, the pair's devices each other's layers (cached
	// grants: the first call pays for them)
	for (int i = 0; i < n; i++) {
		gcmx_ctx* c = slabs[i];
		const bool ok = vmm_grant(c->vmm, lead->device) &&
		                (i == 0 || vmm_grant(c->vmm, slabs[i - 1]->device)) &&
		                (i + 1 == n || vmm_grant(c->vmm, slabs[i + 1]->device));
		if (!ok) return fail(GCMX_ERR_HIP, "peer access to a neighbour's layers refused");
	}
	HIP_TRY(hipSetDevice(lead->device));
	for (int i = 0; i < n; i++) {
		HIP_TRY(hipSetDevice(slabs[i]->device));
		HIP_TRY(hipEventRecord(slabs[i]->ev_ready, slabs[i]->stream));
		HIP_TRY(hipSetDevice(lead->device));
		HIP_TRY(hipStreamWaitEvent(lead->comm_stream, slabs[i]->ev_ready, 0));
	}
	for (int i = 0; i + 1 < n; i++) {
		gcmx_ctx* a = slabs[i];
		gcmx_ctx* b = slabs[i + 1];
		const long long pa = a->geo.stride[0], pb = b->geo.stride[0];
		if (pa != pb) return fail(GCMX_ERR_INVALID_ARG, "slab planes differ");
		const size_t bytes = (size_t)(a->bs * pa) * sizeof(double);
		const int Xa = a->geo.sizes[0];
		for (int comp : a->halo_comps) {
			double* a_plane = a->cur + (size_t)comp * a->geo.cs;
			double* b_plane = b->cur + (size_t)comp * b->geo.cs;
			// a's right ghosts [Xa, Xa+bs) <- b's inner [0, bs)
			HIP_TRY(hipMemcpyPeerAsync(a_plane + (size_t)((Xa + a->bs) * pa), a->device,
			                           b_plane + (size_t)(b->bs * pb), b->device, bytes,
			                           lead->comm_stream));
			// b's left ghosts [-bs, 0) <- a's inner [Xa-bs, Xa)
			HIP_TRY(hipMemcpyPeerAsync(b_plane, b->device, a_plane + (size_t)(Xa * pa), a->device,
			                           bytes, lead->comm_stream));
		}
	}
	HIP_TRY(hipEventRecord(lead->ev_halo, lead->comm_stream));
	for (int i = 0; i < n; i++) {
		HIP_TRY(hipSetDevice(slabs[i]->device));
		HIP_TRY(hipStreamWaitEvent(slabs[i]->stream, lead->ev_halo, 0));
	}
	HIP_TRY(hipSetDevice(lead->device));
	return GCMX_OK;
}

gcmx_status gcmx_comm_init_local(gcmx_ctx* const* ctxs, int n) {
	if (!ctxs || n < 1) return fail(GCMX_ERR_INVALID_ARG, "bad slab list");
	for (int i = 0; i < n; i++) {
		gcmx_ctx* c = ctxs[i];
		if (!c || c->D < 2) return fail(GCMX_ERR_INVALID_ARG, "bad slab (null or dim < 2)");
		if (c->comm || c->lc) return fail(GCMX_ERR_STATE, "communicator already initialised");
		for (int j = 0; j < i; j++)
			if (ctxs[j] == c) return fail(GCMX_ERR_INVALID_ARG, "a context appears twice");
		if (i > 0) {
			const gcmx_ctx* p = ctxs[i - 1];
			bool ok = p->D == c->D && p->bs == c->bs && p->desc.start[0] + p->geo.sizes[0] == c->desc.start[0] &&
			          p->geo.stride[0] == c->geo.stride[0];
			for (int d = 1; d < c->D; d++)
				ok = ok && p->geo.sizes[d] == c->geo.sizes[d] && p->desc.start[d] == c->desc.start[d];
			if (!ok) return fail(GCMX_ERR_INVALID_ARG, "slabs are not X-adjacent with equal y/z extents");
		}
	}
	// neighbours on other devices copy into / out of each other's layers
	for (int i = 0; i + 1 < n; i++)
		if (!vmm_grant(ctxs[i]->vmm, ctxs[i + 1]->device) || !vmm_grant(ctxs[i + 1]->vmm, ctxs[i]->device))
			return fail(GCMX_ERR_HIP, "peer access to a neighbour's layers refused");
	auto L = std::make_shared<LocalComm>();
	L->n = n;
	L->ctx.assign(ctxs, ctxs + n);
	L->posted.assign(n, 0);
	L->issued.assign(n > 1 ? n - 1 : 0, 0);
	for (int t = 0; t < 2; t++) {
		L->issuer[t].assign(n > 1 ? n - 1 : 0, 0);
		L->layer[t].assign(n, nullptr);
		L->ready[t].assign(n, nullptr);
		for (int sd = 0; sd < 2; sd++) L->done[t][sd].assign(n > 1 ? n - 1 : 0, nullptr);
	}
	for (int i = 0; i < n; i++) {
		HIP_TRY(hipSetDevice(ctxs[i]->device));
		for (int t = 0; t < 2; t++) {
			HIP_TRY(hipEventCreateWithFlags(&L->ready[t][i], hipEventDisableTiming));
			// done[t][0][i] is issued by rank i, done[t][1][i-1] by rank i
			if (i + 1 < n) HIP_TRY(hipEventCreateWithFlags(&L->done[t][0][i], hipEventDisableTiming));
			if (i > 0) HIP_TRY(hipEventCreateWithFlags(&L->done[t][1][i - 1], hipEventDisableTiming));
		}
	}
	for (int i = 0; i < n; i++) {
		gcmx_ctx* c = ctxs[i];
		gcmx_status s = halo_wait(c);
		if (s) return s;
		c->lc = L;
		c->lrank = i;
		c->nranks = n;
		c->rank = i;
		c->left = i > 0 ? i - 1 : -1;
		c->right = i + 1 < n ? i + 1 : -1;
		c->halo_gen = 0;
		c->halo_fresh = false;
	}
	HIP_TRY(hipSetDevice(ctxs[0]->device));
	return GCMX_OK;
}

gcmx_status gcmx_local_group_steps(gcmx_ctx* const* ctxs, int n, double tau, int steps) {
	if (!ctxs || n < 1 || steps < 0) return fail(GCMX_ERR_INVALID_ARG, "bad group arguments");
	std::shared_ptr<LocalComm> L = ctxs[0] ? ctxs[0]->lc : nullptr;
	for (int i = 0; i < n; i++)
		if (!ctxs[i] || (n > 1 && (ctxs[i]->lc != L || ctxs[i]->lrank != i)))
			return fail(GCMX_ERR_INVALID_ARG, "contexts are not the ranks of one in-process group, in order");
	std::vector<gcmx_status> st(n, GCMX_OK);
	std::vector<std::string> msg(n);
	auto run = [&](int i) {
		for (int k = 0; k < steps && st[i] == GCMX_OK; k++) st[i] = gcmx_step(ctxs[i], tau);
		if (st[i] == GCMX_OK) st[i] = gcmx_sync(ctxs[i]);
		if (st[i] != GCMX_OK) {
			msg[i] = g_last_error;
			local_abort(ctxs[i], "rank " + std::to_string(i) + ": " + msg[i]);
		}
	};
	std::vector<std::thread> th;
	for (int i = 1; i < n; i++) th.emplace_back(run, i);
	run(0);
	for (auto& t : th) t.join();
	for (int i = 0; i < n; i++)
		if (st[i] != GCMX_OK) return fail(st[i], "rank " + std::to_string(i) + ": " + msg[i]);
	return GCMX_OK;
}

gcmx_status gcmx_sync(gcmx_ctx* c) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (c->lc) {  // the exchange may run on a neighbour's comm stream: wait through the group
		s = halo_wait(c);
		if (s) return s;
	}
	// RCCL: bounded waits (wait_stream) -- a peer that never posts fails the
	// call with GCMX_ERR_COMM instead of hanging it
	if ((s = wait_stream(c, c->comm_stream, "gcmx_sync")) != GCMX_OK ||
	    (s = wait_stream(c, c->inner_stream, "gcmx_sync")) != GCMX_OK ||
	    (s = wait_stream(c, c->bnd_stream, "gcmx_sync")) != GCMX_OK ||
	    (s = wait_stream(c, c->stream, "gcmx_sync")) != GCMX_OK) {
		drain_timings(c);
		return s;
	}
	if (c->halo_pending) {  // the comm stream has drained
		c->halo_pending = false;
		c->halo_fresh = c->halo_layer == c->cur;
	}
	drain_timings(c);
	return GCMX_OK;
}

void* gcmx_stream(gcmx_ctx* c) { return c ? (void*)c->stream : nullptr; }

gcmx_status gcmx_profile_enable(gcmx_ctx* c, int enable) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null context");
	c->prof = enable != 0;
	return GCMX_OK;
}

gcmx_status gcmx_profile_reset(gcmx_ctx* c) {
	gcmx_status s = gcmx_sync(c);
	if (s) return s;
	c->buckets.clear();
	return GCMX_OK;
}

int gcmx_profile_read(gcmx_ctx* c, int index, const char** name, double* total_ms,
                      long long* launches, double* bytes) {
	if (!c) return 0;
	drain_timings(c);
	const int n = (int)c->buckets.size();
	if (index >= 0 && index < n) {
		if (name) *name = c->buckets[index].name.c_str();
		if (total_ms) *total_ms = c->buckets[index].total_ms;
		if (launches) *launches = c->buckets[index].launches;
		if (bytes)
			*bytes = c->buckets[index].launches ? c->buckets[index].bytes / c->buckets[index].launches : 0;
	}
	return n;
}

const char* gcmx_profile_kernel(gcmx_ctx* c, int index) {
	if (!c || index < 0 || index >= (int)c->buckets.size()) return "";
	return c->buckets[index].kernel.c_str();
}

long long gcmx_inner_nodes(gcmx_ctx* c) { return c ? c->geo.n_inner : 0; }
long long gcmx_all_nodes(gcmx_ctx* c) { return c ? c->n_all : 0; }
size_t gcmx_device_bytes(gcmx_ctx* c) { return c ? 2 * c->layer_elems * sizeof(double) : 0; }

}  // extern "C"

namespace {
// The yardstick copy: 16 B per lane, non-temporal stores, 32768 blocks of 256
// threads, grid-stride -- the fastest of the 28 flat-copy shapes tools/copy_probe.hip
// times (1 or 4 or 8 loads in flight per lane, nt or plain stores and loads,
// 1 024-65 536 blocks, grid-stride or one chunk per block: all 4.4-5.2 TB/s on
// the same box, profiles/r3/copy/variants.txt).
typedef double copy_d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_copy_ceiling(const copy_d2* __restrict__ in, copy_d2* __restrict__ out,
                                                      long long n2) {
	const long long stride = (long long)gridDim.x * blockDim.x;
	for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride)
		__builtin_nontemporal_store(in[i], out + i);
}
}  // namespace

extern "C" {

gcmx_status gcmx_copy_ceiling(gcmx_ctx* c, size_t bytes, int reps, float* ms_out) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!ms_out || reps < 1 || bytes < 64) return fail(GCMX_ERR_INVALID_ARG, "bad copy-ceiling arguments");
	const size_t half = bytes / 2 / 16 * 16;
	void *a = nullptr, *b = nullptr;
	// the buffers placed as the layers are (shuffle_policy_mib): one block, a | b
	VmmBlock vb;
	const long long mib = shuffle_policy_mib(2 * half, nullptr);
	if (mib > 0 && vmm_map(c->device, 2 * half, (size_t)mib << 20, vb)) {
		a = vb.va;
		b = static_cast<char*>(vb.va) + half;
	} else if (hipMalloc(&a, half) != hipSuccess || hipMalloc(&b, half) != hipSuccess) {
		if (a) (void)hipFree(a);
		return fail(GCMX_ERR_OOM, "copy-ceiling buffers");
	}
	hipEvent_t e0 = nullptr, e1 = nullptr;
	std::vector<float> ms;
	gcmx_status st = GCMX_OK;
	const long long n2 = (long long)(half / 16);
	if (hipMemsetAsync(a, 0, half, c->stream) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
	    hipEventCreate(&e1) != hipSuccess) {
		st = fail(GCMX_ERR_HIP, "copy-ceiling set-up");
	} else {
		for (int r = 0; r <= reps && st == GCMX_OK; r++) {
			(void)hipEventRecord(e0, c->stream);
			hipLaunchKernelGGL(k_copy_ceiling, dim3(32768), dim3(256), 0, c->stream,
			                   static_cast<const copy_d2*>(a), static_cast<copy_d2*>(b), n2);
			(void)hipEventRecord(e1, c->stream);
			float t = 0.0f;
			if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess)
				st = fail(GCMX_ERR_HIP, "copy-ceiling timing");
			else if (r > 0)  // the first copy warms the buffers' translations
				ms.push_back(t);
		}
	}
	if (e0) (void)hipEventDestroy(e0);
	if (e1) (void)hipEventDestroy(e1);
	if (vb.va) {
		(void)hipStreamSynchronize(c->stream);
		vmm_free(vb);
	} else {
		(void)hipFree(a);
		(void)hipFree(b);
	}
	if (st) return st;
	std::sort(ms.begin(), ms.end());
	*ms_out = ms[ms.size() / 2] * (float)((double)bytes / (double)(2 * half));  // per `bytes`
	return GCMX_OK;
}

gcmx_status gcmx_geometry(gcmx_ctx* c, int64_t out[6]) {
	if (!c || !out) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	const Geo& g = c->geo;
	for (int i = 0; i < 3; i++) out[i] = g.stride[i];
	out[3] = g.cs;
	out[4] = g.origin;
	out[5] = g.row;
	return GCMX_OK;
}

gcmx_status gcmx_layer_info(gcmx_ctx* c, uint64_t out[4]) {
	if (!c || !out) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	out[0] = (uint64_t)(uintptr_t)c->layer_a;
	out[1] = (uint64_t)(uintptr_t)c->layer_b;
	out[2] = (uint64_t)(c->layer_elems * sizeof(double));
	out[3] = c->alloc_kind;
	return GCMX_OK;
}

}  // extern "C"

namespace {
// Clock sampler: ONE wave (lane 0 works) that records (s_memrealtime, s_memtime)
// pairs every `period` ticks of the 100 MHz real-time counter for `span` ticks,
// sleeping in between.  Launched on its own stream before a timed region, it
// shares a CU with whatever runs (it holds 64 threads, no LDS, few VGPRs), so
// Δmemtime / Δrealtime × 100 MHz is the shader clock the chip holds under that
// load (MI355X_MICROARCH.md §DVFS give-back, item 6).  out[0] = samples taken.
__global__ __launch_bounds__(64) void k_clock_probe(unsigned long long* __restrict__ out, int cap,
                                                    unsigned long long period, unsigned long long span) {
	if (threadIdx.x != 0) return;
	const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
	unsigned long long next = r0;
	int n = 0;
	for (int it = 0; it < (1 << 24) && n < cap; it++) {  // bounded: span ends it first
		const unsigned long long r = __builtin_amdgcn_s_memrealtime();
		if (r - r0 > span) break;
		if (r >= next) {
			const unsigned long long t = __builtin_amdgcn_s_memtime();
			out[1 + 2 * n] = r;
			out[2 + 2 * n] = t;
			n++;
			next = r + period;
		}
		__builtin_amdgcn_s_sleep(32);
	}
	out[0] = (unsigned long long)n;
}
}  // namespace

extern "C" {

gcmx_status gcmx_clock_probe_start(gcmx_ctx* c, double seconds, double period_us) {
	gcmx_status s = check_ctx(c);
	if (s) return s;
	if (!(seconds > 0 && seconds <= 30) || !(period_us >= 10))
		return fail(GCMX_ERR_INVALID_ARG, "clock probe: 0 < seconds <= 30, period >= 10 us");
	const int cap = (int)std::min(65536.0, seconds * 1e6 / period_us + 2);
	if (!c->probe_stream) HIP_TRY(hipStreamCreateWithFlags(&c->probe_stream, hipStreamNonBlocking));
	HIP_TRY(hipStreamSynchronize(c->probe_stream));
	if (cap > c->probe_cap) {
		(void)hipFree(c->probe_d);
		c->probe_d = nullptr;
		c->probe_cap = 0;
		HIP_TRY(hipMalloc(&c->probe_d, (1 + 2 * (size_t)cap) * sizeof(unsigned long long)));
		c->probe_cap = cap;
	}
	HIP_TRY(hipMemsetAsync(c->probe_d, 0, sizeof(unsigned long long), c->probe_stream));
	hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, c->probe_stream, c->probe_d, cap,
	                   (unsigned long long)(period_us * 100.0), (unsigned long long)(seconds * 1e8));
	HIP_TRY(hipGetLastError());
	return GCMX_OK;
}

int gcmx_clock_probe_read(gcmx_ctx* c, uint64_t* samples, int cap) {
	if (!c || !c->probe_stream || !c->probe_d) return -1;
	if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->probe_stream) != hipSuccess) return -1;
	unsigned long long n = 0;
	if (hipMemcpy(&n, c->probe_d, sizeof(n), hipMemcpyDeviceToHost) != hipSuccess) return -1;
	const int m = (int)std::min<unsigned long long>(n, (unsigned long long)std::max(cap, 0));
	if (m > 0 && samples &&
	    hipMemcpy(samples, c->probe_d + 1, 2 * (size_t)m * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
	        hipSuccess)
		return -1;
	return (int)n;
}

}  // extern "C"
