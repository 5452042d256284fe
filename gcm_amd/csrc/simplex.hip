// simplex.hip -- device half of the simplex (tetrahedral) grid-characteristic
// stage in Riemann invariants (gsx_* in include/gcmx.h).
//
// One stage s (engine/simplex/Engine.cpp:117-148, GLOBAL_BASIS + PRODUCT):
//   k_sx_transform(U_s)   beforeStage: w = U_s u for every node
//                         (GridCharacteristicMethodInRiemannInvariants.hpp:44-56);
//                         only at the first stage of a step -- later stages get w
//                         from the previous stage's final writers
//   k_sx_gradient         Differentiation::estimateGradient of w (Differentiation.hpp:33-63)
//   k_sx_border           contactAndBorderStage (hpp:57-95) + the border correctors
//                         (applyInGlobalBasis, BorderCorrector.hpp:118-165, 256-265)
//                         + afterStage and the next beforeStage of these nodes
//   k_sx_contact          (multi-body) the contact correctors (ContactCorrector.hpp)
//                         + afterStage / next beforeStage of the contact nodes
//   k_sx_inner            innerStage (hpp:98-112) -- space-time feet read the border
//                         nodes' corrected new invariants -- + afterStage
//                         (u_new = U1_s w_new, hpp:115-126) + next beforeStage; swap.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstring>
#include <string>
#include <memory>
#include <vector>

#include "../../include/gcmx.h"
#include "contact.hpp"
#include "launch.hpp"

namespace {

constexpr int kM = 9;
constexpr int kMaxNb = 20;  // MAX_NUMBER_OF_NEIGHBOR_VERTICES (Cgal3DTriangulation.hpp:53)

gcmx_status fail(gcmx_status s, const std::string& msg) {
	gcmx::set_last_error(msg);
	return s;
}
#define SX_TRY(expr)                                                                   \
	do {                                                                               \
		hipError_t e_ = (expr);                                                        \
		if (e_ != hipSuccess)                                                          \
			return fail(GCMX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
	} while (0)

// Every kernel launch on a context's stream, counted (gsx_launch_count: the
// dependent launches of a step, for its launch-floor model).
#define SX_LAUNCH(ctx, ...)                \
	do {                                   \
		++(ctx)->launches;                 \
		hipLaunchKernelGGL(__VA_ARGS__);   \
	} while (0)

struct BorderArgs {  // static per-condition data passed by value with every launch
	int type[GSX_MAX_BORDER_CONDITIONS];
	double minDet[GSX_MAX_BORDER_CONDITIONS][3];
	const double* b;  // device [condition][3]: b(t) of the step, written per step
};

struct BorderDev {
	int n = 0, nCond = 0;
	int *nodes = nullptr, *cond = nullptr;
	double *B = nullptr, *S = nullptr;
	signed char* outer = nullptr;
	double* md = nullptr;  // [entry][stage][side R, L][10]: B * Omega (3x3) and det, k_sx_border_prep
	int2* nodeRec = nullptr;  // [node]: (plan entry, its condition) or (-1, 0)
	BorderArgs args{};
	BorderArgs* argsDev = nullptr;  // device copy of args (what the kernels read)
	bool set = false, valuesSet = false;
	double lastValues[3 * GSX_MAX_BORDER_CONDITIONS] = {};  // what bvals holds once valuesSet
};

struct StageShift {  // crossingPoints' shift of every invariant: direction * (-tau L(k))
	double d[6][3];
};

// Feet in a compact, coalesced layout ([k][pos], pos = position in the stage's
// border list, then its inner list): fv = the cell's (or face's)
// vertices, flam = barycentric weights, fmeta = kind | slot(i) << (4 + 4 i).  The
// foot point of a CELL foot is recomputed as coords[n] + shift[k], the same IEEE
// sum the host's plan made (gsx_set_stage_plan checks it).
struct StageDev {
	int4* fv = nullptr;
	double4* flam = nullptr;
	int* fmeta = nullptr;
	StageShift shift{};
	int* border = nullptr;
	int* inner = nullptr;
	int nBorder = 0, nInner = 0;
	bool set = false;
	// every new-invariant (wn) read of an inner foot names a node of this stage's
	// border list, and no border foot reads wn: the stage may run as one launch
	// (k_sx_stage_l8) whose inner groups wait for exactly those border nodes
	bool fusable = false;
	int waitFeet = 0;  // inner feet that wait for border nodes in the one-launch stage
	// border corrector records by position t in `border` (k_sx_border_rec): plan
	// entry, condition, outer code, which sides are solvable; B; B * Omega and det
	int4* rec = nullptr;
	double *recB = nullptr, *recMd = nullptr;
};

}  // namespace

struct gsx_ctx {
	int device = 0, N = 0;
	hipStream_t stream = nullptr;
	std::vector<double> hostCoords;  // [n][3]
	double *coords = nullptr, *u = nullptr, *un = nullptr, *w = nullptr, *wn = nullptr,
	       *grad = nullptr;
	double* arena = nullptr;  // one allocation holding u, un, w, wn, grad, wnext
	double* mats = nullptr;  // [2][3][81]: U then U1
	bool matsSet = false;
	int nodeLanes = 0;  // gsx_set_node_lanes: 0 auto, 1, 8
	int *gOff = nullptr, *gNb = nullptr;
	double *gRows = nullptr, *gW = nullptr, *gM = nullptr, *gDet = nullptr;
	bool gradSet = false;
	StageDev st[3];
	BorderDev bd;
	double* wnext = nullptr;             // next stage's invariants, node-major [n][9]
	int wStage = -1;                     // w already holds the invariants of this stage (-1: none)
	int* corrOf = nullptr;               // node -> border-plan entry or -1
	char* deferred = nullptr;            // node in a contact: the contact kernel finalizes it
	std::vector<char> hostDeferred;
	double* bvals = nullptr;             // [GSX_MAX_BORDER_CONDITIONS][3] border values b(t)
	std::unique_ptr<struct StepGraphs> graphs;  // gsx_step's replayed steps (this ctx leads)
	unsigned planGen = 0;  // bumped by every call that (re)sets device plan data graphs point into
	// one-launch stages (gsx_stage, eight-lane layout): per-node "wn written in
	// launch #epoch" flags [N], the finished-gradient-block counter, then one error
	// word (a wait that timed out)
	int* ready = nullptr;
	int epoch = 0;
	unsigned gTarget = 0;
	unsigned tickets = 0;  // work tickets k_sx_stage_l8 launches have handed out (device counter ready[N + 2])
	long long launches = 0;  // kernel launches on this context's stream (gsx_launch_count)
	int fuseMode = 1;  // gsx_set_stage_fusion: 0 never, 1 border + inner, 2 gradient + border + inner,
	                   // 3 border + inner without the grid-size cap (tuning)
	bool lastFused = false;  // the last gsx_stage ran as one launch
	int waitBudget = 1 << 20;  // polls per device wait (gsx_set_wait_budget)
};

// The host-side state a simplex step changes (pointer swaps, chaining flag).
struct BodyState {
	double *u, *un, *w, *wnext;
	int wStage;
	bool operator==(const BodyState& o) const {
		return u == o.u && un == o.un && w == o.w && wnext == o.wnext && wStage == o.wStage;
	}
};
static BodyState body_state(const gsx_ctx* c) { return {c->u, c->un, c->w, c->wnext, c->wStage}; }
static void set_body_state(gsx_ctx* c, const BodyState& b) {
	c->u = b.u;
	c->un = b.un;
	c->w = b.w;
	c->wnext = b.wnext;
	c->wStage = b.wStage;
}

// One captured step per entry state: a step swaps u/un, so two graphs alternate.
struct StepGraphs {
	std::vector<gsx_ctx*> bodies;
	std::vector<gsx_contact*> contacts;
	std::vector<unsigned> gens;  // the bodies' planGen at capture
	struct Entry {
		std::vector<BodyState> before, after;
		hipGraph_t graph = nullptr;
		hipGraphExec_t exec = nullptr;
	};
	std::vector<Entry> entries;
	hipEvent_t evFork = nullptr, evJoin = nullptr;
	std::vector<hipEvent_t> evBody;
	~StepGraphs() {
		for (auto& e : entries) {
			if (e.exec) (void)hipGraphExecDestroy(e.exec);
			if (e.graph) (void)hipGraphDestroy(e.graph);
		}
		if (evFork) (void)hipEventDestroy(evFork);
		if (evJoin) (void)hipEventDestroy(evJoin);
		for (hipEvent_t e : evBody) (void)hipEventDestroy(e);
	}
};

struct gsx_contact {
	gsx_ctx *a = nullptr, *b = nullptr;
	int n = 0;
	int *na = nullptr, *nb = nullptr;
	double *normal = nullptr, *S = nullptr;
	signed char *codeA = nullptr, *codeB = nullptr;
	double minDet[3][2] = {};
	hipEvent_t evA = nullptr, evB = nullptr;
};

namespace {

// Global thread index with the blocks of each XCD made contiguous: workgroups
// are dealt round-robin over the 8 XCDs (b % 8, MI355X_MICROARCH.md §Workgroup
// dispatch), so XCD k gets blocks k, k+8, ...; renumbering them k*q + min(k, r)
// + b/8 hands XCD k one contiguous range of nodes, whose neighbours / cell
// vertices (spatially close in the vertex order) its own L2 then holds.  For
// kernels whose blocks are independent only (not k_sx_stage_l8, whose waits
// rely on block id order).
__device__ __forceinline__ int xcd_gid() {
	const int T = (int)gridDim.x, b = (int)blockIdx.x, q = T >> 3, r = T & 7, k = b & 7;
	return (k * q + (k < r ? k : r) + (b >> 3)) * (int)blockDim.x + (int)threadIdx.x;
}

// out[c] = M(c,0) in[0] + sum_{j>=1} M(c,j) in[j]  (linal/operators.hpp:109-123).
// AOS_OUT: the invariants of beforeStage are written node-major ([n][9]) because
// the gradient and node kernels gather them per neighbour / per cell vertex.
template <bool AOS_OUT>
__global__ __launch_bounds__(256) void k_sx_transform(const double* __restrict__ in,
                                                      double* __restrict__ out,
                                                      const double* __restrict__ Mx, int N) {
	const int n = xcd_gid();
	if (n >= N) return;
	double v[kM];
#pragma unroll
	for (int j = 0; j < kM; j++) v[j] = in[j * N + n];
#pragma unroll
	for (int c = 0; c < kM; c++) {
		double s = Mx[c * kM + 0] * v[0];
#pragma unroll
		for (int j = 1; j < kM; j++) s += Mx[c * kM + j] * v[j];
		if (AOS_OUT) out[(size_t)n * kM + c] = s;
		else out[c * N + n] = s;
	}
}

__device__ __forceinline__ double det3(double m11, double m12, double m13, double m21, double m22,
                                       double m23, double m31, double m32, double m33) {
	return m11 * (m22 * m33 - m23 * m32) - m12 * (m21 * m33 - m23 * m31) +
	       m13 * (m21 * m32 - m22 * m31);
}

// linearLeastSquares(A, b, W) = solve(A^T W A, A^T (W b)) per component, with
// transposeMultiply's order (first term, then +=) over all kMaxNb rows: the
// unused rows are zero rows and add +0.  Neighbour-outer loop: each neighbour's
// weight and its invariants (one node-major record) are read once; every
// component still sums its terms in neighbour order.  The LSQ row is the same
// IEEE difference coords[neighbour] - coords[node] the host plan made
// (gsx_set_gradient_plan checks it).  Only invariants 0..5 get gradients: the
// zero-eigenvalue invariants 6..8 are exact hits and never interpolated
// (hpp:166-170).  w is node-major [n][9], grad [n][3][6].
constexpr int kG = 6;
__global__ __launch_bounds__(256) void k_sx_gradient(const double* __restrict__ w,
                                                     double* __restrict__ grad,
                                                     const int* __restrict__ off,
                                                     const int* __restrict__ nbs,
                                                     const double* __restrict__ coords,
                                                     const double* __restrict__ wts,
                                                     const double* __restrict__ Mm,
                                                     const double* __restrict__ dets, int N) {
	const int n = xcd_gid();
	if (n >= N) return;
	const int b0 = off[n], K = off[n + 1] - b0;
	double wc[kG], r0[kG], r1[kG], r2[kG];
#pragma unroll
	for (int c = 0; c < kG; c++) wc[c] = w[(size_t)n * kM + c];
	const double x0 = coords[3 * (size_t)n], x1 = coords[3 * (size_t)n + 1],
	             x2 = coords[3 * (size_t)n + 2];
	// Latency layout: all neighbour indices in one round trip, then the
	// neighbours' records in batches of kGB (their loads issued together); the
	// sums still run in neighbour order.
	constexpr int kGB = 5;
	int nbv[kMaxNb];
#pragma unroll
	for (int i = 0; i < kMaxNb; i++) nbv[i] = i < K ? nbs[b0 + i] : n;
#pragma unroll
	for (int i0 = 0; i0 < kMaxNb; i0 += kGB) {
		if (i0 >= K) break;
		double wb_[kGB][kG], a_[kGB][3], we_[kGB];
#pragma unroll
		for (int j = 0; j < kGB; j++) {
			const int nb = nbv[i0 + j];
			const double* wn = w + (size_t)nb * kM;
#pragma unroll
			for (int c = 0; c < kG; c++) wb_[j][c] = wn[c];
#pragma unroll
			for (int r = 0; r < 3; r++) a_[j][r] = coords[3 * (size_t)nb + r];
			we_[j] = i0 + j < K ? wts[b0 + i0 + j] : 0.0;
		}
#pragma unroll
		for (int j = 0; j < kGB; j++) {
			const int i = i0 + j;
			if (i < K) {
				const double a0 = a_[j][0] - x0, a1 = a_[j][1] - x1, a2 = a_[j][2] - x2;
				const double we = we_[j];
#pragma unroll
				for (int c = 0; c < kG; c++) {
					const double bi = wb_[j][c] - wc[c];  // b(i) = pde(neighbor) - pde(it)
					const double wb = we * bi;            // (W * b)(i)
					const double t0 = a0 * wb, t1 = a1 * wb, t2 = a2 * wb;
					if (i == 0) {
						r0[c] = t0; r1[c] = t1; r2[c] = t2;
					} else {
						r0[c] += t0; r1[c] += t1; r2[c] += t2;
					}
				}
			}
		}
	}
	const double* M = Mm + 9 * (size_t)n;
	const double det = dets[n];
	const double m0 = M[0], m1 = M[1], m2 = M[2], m3 = M[3], m4 = M[4], m5 = M[5], m6 = M[6],
	             m7 = M[7], m8 = M[8];
	double* g = grad + (size_t)n * 3 * kG;
#pragma unroll
	for (int c = 0; c < kG; c++) {
		double y0 = r0[c], y1 = r1[c], y2 = r2[c];
		if (K < kMaxNb) {  // the zero rows: 0 * (0 * 0) = +0
			y0 += 0.0; y1 += 0.0; y2 += 0.0;
		}
		const double d1 = det3(y0, m1, m2, y1, m4, m5, y2, m7, m8);
		const double d2 = det3(m0, y0, m2, m3, y1, m5, m6, y2, m8);
		const double d3 = det3(m0, m1, y0, m3, m4, y1, m6, m7, y2);
		g[0 * kG + c] = d1 / det;
		g[1 * kG + c] = d2 / det;
		g[2 * kG + c] = d3 / det;
	}
}

__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

// interpolateValuesAround (hpp:156-198) for the listed nodes, feet resolved on the host.
// Latency layout: the six feet's records are read first, then every foot's
// gathers are issued without branches (all foot vertex indices are valid nodes,
// gsx_set_stage_plan checks them; a foot that needs no gradient still reads one
// it ignores), so one node costs three dependent memory round trips, not three
// per foot.  The arithmetic of the selected kind is unchanged.
__device__ __forceinline__ void node_invariants(int n, int pos, int P, const int4* __restrict__ fv,
                                                const double4* __restrict__ flam,
                                                const int* __restrict__ fmeta, const StageShift& sh,
                                                const double* __restrict__ coords,
                                                const double* __restrict__ w,
                                                const double* __restrict__ grad,
                                                const double* __restrict__ wn, int N,
                                                double (&out)[kM]) {
	const double x0 = coords[3 * (size_t)n + 0], x1 = coords[3 * (size_t)n + 1],
	             x2 = coords[3 * (size_t)n + 2];
	int meta[6];
	int4 fvv[6];
	double4 lv[6];
#pragma unroll
	for (int k = 0; k < 6; k++) {
		const size_t e = (size_t)k * P + pos;
		meta[k] = fmeta[e];
		fvv[k] = fv[e];
		lv[k] = flam[e];
	}
#pragma unroll
	for (int k = 6; k < kM; k++) out[k] = w[(size_t)n * kM + k];  // dx(k) == 0: exact hit (hpp:166-170)
#pragma unroll
	for (int k = 0; k < 6; k++) {
		const int kind = meta[k] & 15;
		const int vs[4] = {fvv[k].x, fvv[k].y, fvv[k].z, fvv[k].w};
		const double lam[4] = {lv[k].x, lv[k].y, lv[k].z, lv[k].w};
		double v[4], term[4];
		const double q0 = x0 + sh.d[k][0], q1 = x1 + sh.d[k][1], q2 = x2 + sh.d[k][2];
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const int p = vs[i];
			// SPACETIME: value i is slot s of the face's current (s < 3) or new (s >= 3) invariants
			const int sl = (meta[k] >> (4 + 4 * i)) & 15;
			const int r = sl < 3 ? sl : sl - 3;
			const int ps = r == 0 ? vs[0] : (r == 1 ? vs[1] : vs[2]);
			const double* src = (kind == GSX_FOOT_CELL) ? w + (size_t)p * kM + k
			                    : (sl < 3)              ? w + (size_t)ps * kM + k
			                                            : wn + (size_t)ps * kM + k;
			v[i] = *src;
			// TetrahedronInterpolator::hybridInterpolate (hpp:93-104) terms
			const double d0 = q0 - coords[3 * (size_t)p + 0];
			const double d1 = q1 - coords[3 * (size_t)p + 1];
			const double d2 = q2 - coords[3 * (size_t)p + 2];
			const double* gp = grad + (size_t)p * 3 * kG;
			double dot = gp[0 * kG + k] * d0;
			dot += gp[1 * kG + k] * d1;
			dot += gp[2 * kG + k] * d2;
			term[i] = v[i] + dot / 2.0;
		}
		double ans;
		if (kind == GSX_FOOT_CELL) {
			const double quadratic =
			    lam[0] * term[0] + lam[1] * term[1] + lam[2] * term[2] + lam[3] * term[3];
			const double mn = std_min(std_min(std_min(v[0], v[1]), v[2]), v[3]);
			const double mx = std_max(std_max(std_max(v[0], v[1]), v[2]), v[3]);
			const double limited = std_min(std_max(quadratic, mn), mx);
			ans = (quadratic == limited) ? quadratic
			                             : lam[0] * v[0] + lam[1] * v[1] + lam[2] * v[2] + lam[3] * v[3];
		} else if (kind == GSX_FOOT_SPACETIME) {
			// the face's border nodes: current invariants w, new invariants wn
			ans = lam[0] * v[0] + lam[1] * v[1] + lam[2] * v[2] + lam[3] * v[3];
		} else {
			ans = 0.0;  // outer invariant / walk ended on a vertex
		}
		out[k] = ans;
	}
}

// Symmetric-storage slot of sigma(i, j) in the PDE vector (linal/Symmetry.hpp:38-46,
// VelocitySigmaVariables.hpp:82-96): Vx Vy Vz Sxx Sxy Sxz Syy Syz Szz.
__device__ __forceinline__ int sym(int i, int j) {
	const int a = i < j ? i : j, b = i < j ? j : i;
	return 3 + a * 3 - ((a - 1) * a) / 2 + b - a;
}

// ElasticModel::applyPlainBorderCorrection (ElasticModel.hpp:202-228) on one PDE vector.
__device__ void plain_correction(double (&u)[kM], int type, const double* __restrict__ S,
                                 const double (&b)[3]) {
	if (type == GSX_FIXED_FORCE) {
		double sg[3][3], t[3][3], sl[3][3];
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) sg[i][j] = u[sym(i, j)];  // getSigmaFrom
		for (int i = 0; i < 3; i++)  // S_T * sigmaGlobal
			for (int j = 0; j < 3; j++) {
				double x = S[0 * 3 + i] * sg[0][j];
				x += S[1 * 3 + i] * sg[1][j];
				x += S[2 * 3 + i] * sg[2][j];
				t[i][j] = x;
			}
		for (int i = 0; i < 3; i++)  // (...) * S
			for (int j = 0; j < 3; j++) {
				double x = t[i][0] * S[0 * 3 + j];
				x += t[i][1] * S[1 * 3 + j];
				x += t[i][2] * S[2 * 3 + j];
				sl[i][j] = x;
			}
		for (int i = 0; i < 3; i++) sl[i][2] = b[i];  // setColumn(D - 1, value)
		for (int j = 0; j < 3; j++) sl[2][j] = b[j];  // setRow(D - 1, value)
		for (int i = 0; i < 3; i++)  // S * sigmaLocal
			for (int j = 0; j < 3; j++) {
				double x = S[i * 3 + 0] * sl[0][j];
				x += S[i * 3 + 1] * sl[1][j];
				x += S[i * 3 + 2] * sl[2][j];
				t[i][j] = x;
			}
		for (int i = 0; i < 3; i++)  // (...) * S_T, then setSigmaTo (row-major writes)
			for (int j = 0; j < 3; j++) {
				double x = t[i][0] * S[j * 3 + 0];
				x += t[i][1] * S[j * 3 + 1];
				x += t[i][2] * S[j * 3 + 2];
				u[sym(i, j)] = x;
			}
	} else {
		for (int i = 0; i < 3; i++) {  // velocity = S * value
			double x = S[i * 3 + 0] * b[0];
			x += S[i * 3 + 1] * b[1];
			x += S[i * 3 + 2] * b[2];
			u[i] = x;
		}
	}
}

// calculateOuterWaveCorrection (common.hpp:186-202) with Omega = the U1 columns
// `cols` (getColumnsFromGcmMatrices, common.hpp:153-165).
// Its matrix part, B * Omega and det, depends only on the node's border matrix and
// the stage's U1: owc_matrix is what k_sx_border_prep evaluates once per plan.
template <class BT>  // B: a pointer into the plan or the node's 27 values in registers
__device__ __forceinline__ double owc_matrix(const double* __restrict__ U1, const int (&cols)[3],
                                             const BT& B, double (&M)[3][3]) {
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) {
			double x = B[i * kM + 0] * U1[0 * kM + cols[j]];
			for (int n = 1; n < kM; n++) x += B[i * kM + n] * U1[n * kM + cols[j]];
			M[i][j] = x;
		}
	return det3(M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2], M[2][0], M[2][1], M[2][2]);
}

template <class BT>  // B: a pointer into the plan or the node's 27 values in registers
__device__ bool outer_wave_correction(const double (&u)[kM], const double* __restrict__ U1,
                                      const int (&cols)[3], const BT& B,
                                      const double (&b)[3], double minValid, double (&value)[kM]) {
	double M[3][3];
	const double det = owc_matrix(U1, cols, B, M);
	if (!(fabs(det) > minValid)) return false;
	double r[3];
	for (int i = 0; i < 3; i++) {
		double x = B[i * kM + 0] * u[0];
		for (int n = 1; n < kM; n++) x += B[i * kM + n] * u[n];
		r[i] = b[i] - x;
	}
	// linal::solveLinearSystem 3x3 (linearSystems.hpp:104-129)
	const double d1 = det3(r[0], M[0][1], M[0][2], r[1], M[1][1], M[1][2], r[2], M[2][1], M[2][2]);
	const double d2 = det3(M[0][0], r[0], M[0][2], M[1][0], r[1], M[1][2], M[2][0], r[2], M[2][2]);
	const double d3 = det3(M[0][0], M[0][1], r[0], M[1][0], M[1][1], r[1], M[2][0], M[2][1], r[2]);
	const double alpha[3] = {d1 / det, d2 / det, d3 / det};
	for (int i = 0; i < kM; i++) {
		double x = U1[i * kM + cols[0]] * alpha[0];
		x += U1[i * kM + cols[1]] * alpha[1];
		x += U1[i * kM + cols[2]] * alpha[2];
		value[i] = x;
	}
	return true;
}

__device__ __forceinline__ void mat_vec(const double* __restrict__ Mx, const double (&in)[kM],
                                        double (&out)[kM]) {
#pragma unroll
	for (int c = 0; c < kM; c++) {
		double s = Mx[c * kM + 0] * in[0];
#pragma unroll
		for (int j = 1; j < kM; j++) s += Mx[c * kM + j] * in[j];
		out[c] = s;
	}
}

// BorderCorrectorInRiemannInvariants::applyInGlobalBasis (BorderCorrector.hpp:256-265)
// on one node's new invariants w: -> PDE (U1), BorderCorrectorInPdeVectors::
// applyInGlobalBasis (:118-165), -> invariants (U).  t = the node's border-plan entry.
__device__ void border_correct(double (&w)[kM], int t, const int* __restrict__ cond,
                               const double* __restrict__ Bm, const double* __restrict__ Sm,
                               const signed char* __restrict__ outer, int count,
                               const double* __restrict__ U, const double* __restrict__ U1,
                               int stage, const BorderArgs& args) {
	const int c = cond[t];
	const int code = outer[(size_t)stage * count + t];
	const double* B = Bm + 27 * (size_t)t;
	const double b[3] = {args.b[3 * c], args.b[3 * c + 1], args.b[3 * c + 2]};
	const double minValid = args.minDet[c][stage];
	double u[kM];
	mat_vec(U1, w, u);
	const int R[3] = {1, 3, 5}, L[3] = {0, 2, 4};  // Model.cpp:81-82
	if (code == 1 || code == 2) {
		double v[kM];
		if (outer_wave_correction(u, U1, code == 1 ? R : L, B, b, minValid, v)) {
			for (int k = 0; k < kM; k++) u[k] += v[k];
		} else {
			plain_correction(u, args.type[c], Sm + 9 * (size_t)t, b);
		}
	} else {
		// double-outer or fully inner: average of both sides (:146-162)
		double vr[kM], vl[kM];
		const bool okR = outer_wave_correction(u, U1, R, B, b, minValid, vr);
		const bool okL = outer_wave_correction(u, U1, L, B, b, minValid, vl);
		if (okR && okL) {
			for (int k = 0; k < kM; k++) u[k] += (vr[k] + vl[k]) / 2;
		} else {
			plain_correction(u, args.type[c], Sm + 9 * (size_t)t, b);
		}
	}
	mat_vec(U, u, w);
}

// afterStage for one node (u_new = U1_s w_new, hpp:115-126) and, when the next
// stage of the step follows, its beforeStage (w' = U_{s+1} u_new, node-major):
// the node's final writer does both, so no separate transform pass is needed.
__device__ __forceinline__ void finalize(int n, const double (&wv)[kM], const double* __restrict__ U1,
                                         const double* __restrict__ Unext, double* __restrict__ un,
                                         double* __restrict__ wnext, int N) {
	double u[kM];
	mat_vec(U1, wv, u);
#pragma unroll
	for (int k = 0; k < kM; k++) un[k * N + n] = u[k];
	if (Unext) {
		double w2[kM];
		mat_vec(Unext, u, w2);
#pragma unroll
		for (int k = 0; k < kM; k++) wnext[(size_t)n * kM + k] = w2[k];
	}
}

struct BorderDevArgs {  // the border plan's device arrays (null cond = no plan)
	const int *corrOf, *cond;
	const double *B, *S;
	const signed char* outer;
	int count, ncond;
	const int4* rec;  // the stage's corrector records by list position (eight-lane kernel)
	const double *recB, *recMd;
};

// contactAndBorderStage (hpp:57-95) for the contact and border nodes, the border
// correctors of the border-plan nodes inline (BorderCorrector.hpp:118-165: they
// only read the node's own new invariants) and, for every node that is not in a
// contact, afterStage + the next beforeStage.  wn keeps the corrected invariants
// of these nodes: inner space-time feet and the contact correctors read them.
// The corrector kernels read U / U1 / U_next entry by entry in long unrolled
// sums; as uniform loads they land in SGPRs, which overflow into VGPR lanes (1 200+
// v_readlane per launch, measured 10 us of a 19 us border launch at 16^3).  Staged
// once per block in LDS, every entry is a broadcast ds_read instead.
template <int NMAT>
struct SharedMats {
	double m[NMAT][81];
};
template <int NMAT>
__device__ __forceinline__ void stage_mats(SharedMats<NMAT>& sm, const double* const (&src)[NMAT]) {
	for (int i = threadIdx.x; i < 81; i += blockDim.x)
#pragma unroll
		for (int k = 0; k < NMAT; k++)
			if (src[k]) sm.m[k][i] = src[k][i];
	__syncthreads();
}

__global__ __launch_bounds__(64) void k_sx_border(
    const int* __restrict__ nodes, int count, const int4* __restrict__ fv,
    const double4* __restrict__ flam, const int* __restrict__ fmeta, StageShift sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    double* __restrict__ wn, const char* __restrict__ deferred, BorderDevArgs bp, const BorderArgs* __restrict__ argp,
    const double* __restrict__ U, const double* __restrict__ U1, const double* __restrict__ Unext,
    double* __restrict__ un, double* __restrict__ wnext, int stage, int N, int pos0, int P) {
	const BorderArgs& args = *argp;  // static per plan: device memory, not kernel arguments
	__shared__ SharedMats<3> sm;
	stage_mats<3>(sm, {U, U1, Unext});
	const int t = xcd_gid();
	if (t >= count) return;
	const int n = nodes[t];
	double out[kM];
	node_invariants(n, pos0 + t, P, fv, flam, fmeta, sh, coords, w, grad, wn, N, out);
	if (bp.cond) {
		const int ci = bp.corrOf[n];
		if (ci >= 0)
			border_correct(out, ci, bp.cond, bp.B, bp.S, bp.outer, bp.count, sm.m[0], sm.m[1], stage, args);
	}
#pragma unroll
	for (int k = 0; k < kM; k++) wn[(size_t)n * kM + k] = out[k];
	if (!deferred[n]) finalize(n, out, sm.m[1], Unext ? sm.m[2] : nullptr, un, wnext, N);
}

// innerStage (hpp:98-112) + afterStage + the next beforeStage for the inner nodes;
// space-time feet read the border nodes' corrected new invariants (wn).
__global__ __launch_bounds__(256) void k_sx_inner(
    const int* __restrict__ nodes, int count, const int4* __restrict__ fv,
    const double4* __restrict__ flam, const int* __restrict__ fmeta, StageShift sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    const double* __restrict__ wn, const double* __restrict__ U1, const double* __restrict__ Unext,
    double* __restrict__ un, double* __restrict__ wnext, int N, int pos0, int P) {
	const int t = xcd_gid();
	if (t >= count) return;
	const int n = nodes[t];
	double out[kM];
	node_invariants(n, pos0 + t, P, fv, flam, fmeta, sh, coords, w, grad, wn, N, out);
	finalize(n, out, U1, Unext, un, wnext, N);
}

// ---- latency layout: eight lanes per node (gsx_set_node_lanes) ----------------
// Small meshes (the reference's 16^3 cube: 4 913 nodes) leave most of the chip
// idle with one thread per node, and a node's work is a chain of dependent
// gathers.  Here lane c of a node's group of kL handles component / foot c: the
// gradient lanes sum their own component's terms (in neighbour order, as the
// node-per-thread kernel), the foot lanes interpolate their own invariant, and
// the 9 results meet through cross-lane shuffles (__shfl within the group); the
// U1 / U products are split by rows.  Every value is produced by the same
// operations in the same order as in the node-per-thread kernels.
constexpr int kL = 8;
// Threads per block of the eight-lane kernels: their launches are a few thousand
// groups of gather chains, so small blocks spread them over more CUs (each CU's
// L1 / address units serve fewer gathering waves).
#ifndef GCMX_SX_L8_BLOCK
#define GCMX_SX_L8_BLOCK 256
#endif
constexpr int kL8Block = GCMX_SX_L8_BLOCK;
// Automatic node-kernel layout: eight lanes per node below this many vertices.
constexpr int kL8MaxNodes = 131072;
// Largest one-launch stage (k_sx_stage_l8), in blocks.  Measured (one box,
// profiles/r2/simplex_fused/f64.txt): 32^3 meshes (1 120 blocks) gain 14-8 %
// against two launches, 64^3 (8 600 blocks) lose 11 % on the cube.
constexpr size_t kFuseMaxBlocks = 4096;

template <bool SC1>
__device__ __forceinline__ void gradient_node_l8(int gid, const double* __restrict__ w, double* __restrict__ grad,
                                                 const int* __restrict__ off, const int* __restrict__ nbs,
                                                 const double* __restrict__ coords, const double* __restrict__ wts,
                                                 const double* __restrict__ Mm, const double* __restrict__ dets,
                                                 int N) {
	const int n = gid / kL, c = gid % kL;
	if (n >= N || c >= kG) return;  // no shuffles in this kernel
	const int b0 = off[n], K = off[n + 1] - b0;
	const double wc = w[(size_t)n * kM + c];
	const double x0 = coords[3 * (size_t)n], x1 = coords[3 * (size_t)n + 1],
	             x2 = coords[3 * (size_t)n + 2];
	constexpr int kGB = 10;
	int nbv[kMaxNb];
#pragma unroll
	for (int i = 0; i < kMaxNb; i++) nbv[i] = i < K ? nbs[b0 + i] : n;
	double r0 = 0.0, r1 = 0.0, r2 = 0.0;
#pragma unroll
	for (int i0 = 0; i0 < kMaxNb; i0 += kGB) {
		if (i0 >= K) break;
		double wb_[kGB], a_[kGB][3], we_[kGB];
#pragma unroll
		for (int j = 0; j < kGB; j++) {
			const int nb = nbv[i0 + j];
			wb_[j] = w[(size_t)nb * kM + c];
#pragma unroll
			for (int r = 0; r < 3; r++) a_[j][r] = coords[3 * (size_t)nb + r];
			we_[j] = i0 + j < K ? wts[b0 + i0 + j] : 0.0;
		}
#pragma unroll
		for (int j = 0; j < kGB; j++) {
			const int i = i0 + j;
			if (i < K) {
				const double a0 = a_[j][0] - x0, a1 = a_[j][1] - x1, a2 = a_[j][2] - x2;
				const double bi = wb_[j] - wc;  // b(i) = pde(neighbor) - pde(it)
				const double wb = we_[j] * bi;  // (W * b)(i)
				const double t0 = a0 * wb, t1 = a1 * wb, t2 = a2 * wb;
				if (i == 0) {
					r0 = t0; r1 = t1; r2 = t2;
				} else {
					r0 += t0; r1 += t1; r2 += t2;
				}
			}
		}
	}
	const double* M = Mm + 9 * (size_t)n;
	const double det = dets[n];
	double y0 = r0, y1 = r1, y2 = r2;
	if (K < kMaxNb) {  // the zero rows: 0 * (0 * 0) = +0
		y0 += 0.0; y1 += 0.0; y2 += 0.0;
	}
	const double d1 = det3(y0, M[1], M[2], y1, M[4], M[5], y2, M[7], M[8]);
	const double d2 = det3(M[0], y0, M[2], M[3], y1, M[5], M[6], y2, M[8]);
	const double d3 = det3(M[0], M[1], y0, M[3], M[4], y1, M[6], M[7], y2);
	double* g = grad + (size_t)n * 3 * kG;
	if constexpr (SC1) {  // handed off inside the launch: write-through
		__hip_atomic_store(g + 0 * kG + c, d1 / det, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		__hip_atomic_store(g + 1 * kG + c, d2 / det, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		__hip_atomic_store(g + 2 * kG + c, d3 / det, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	} else {
		g[0 * kG + c] = d1 / det;
		g[1 * kG + c] = d2 / det;
		g[2 * kG + c] = d3 / det;
	}
}

// SIGNAL: count the block once all its gradients are stored (k_sx_stage_l8).
template <bool SIGNAL>
__device__ __forceinline__ void gradient_l8(int gid, const double* __restrict__ w, double* __restrict__ grad,
                                            const int* __restrict__ off, const int* __restrict__ nbs,
                                            const double* __restrict__ coords, const double* __restrict__ wts,
                                            const double* __restrict__ Mm, const double* __restrict__ dets, int N,
                                            unsigned* __restrict__ gcount) {
	gradient_node_l8<SIGNAL>(gid, w, grad, off, nbs, coords, wts, Mm, dets, N);
	if constexpr (SIGNAL) {  // every storing wave drains its sc1 stores, then one lane counts the block
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		if (threadIdx.x == 0) __hip_atomic_fetch_add(gcount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}

__global__ __launch_bounds__(256) void k_sx_gradient_l8(const double* __restrict__ w,
                                                        double* __restrict__ grad,
                                                        const int* __restrict__ off,
                                                        const int* __restrict__ nbs,
                                                        const double* __restrict__ coords,
                                                        const double* __restrict__ wts,
                                                        const double* __restrict__ Mm,
                                                        const double* __restrict__ dets, int N) {
	gradient_l8<false>(xcd_gid(), w, grad, off, nbs, coords, wts, Mm, dets, N, nullptr);
}

// A border node's new invariants (wn) are complete once its flag holds this
// launch's epoch (k_sx_stage_l8).  Bounded: a wait that cannot end (a plan the
// host check missed) sets the error word instead of hanging the device.
struct StageWait {
	int* ready;         // [N] border nodes' wn stored (== epoch)
	unsigned* gcount;   // gradient blocks finished, monotonic
	unsigned gtarget;   // gcount once this launch's gradient blocks are done
	int epoch;
	int* err;
	int budget;         // polls before a wait gives up (gsx_set_wait_budget; < 0: every wait reports a timeout)
	unsigned* ticket;   // work tickets handed out, monotonic (k_sx_stage_l8)
	unsigned tbase;     // *ticket when this launch started
};
// Hand-offs inside k_sx_stage_l8 (cdna_hip_programming.md Guideline 16, the
// write-through form): every handed-off byte (gradients, wn) is stored sc1 by its
// producer wave, which drains its stores (vmcnt(0)) before the flag / counter is
// written by an atomic; every load of those bytes is an sc1 load (read_ready), so
// the consumer needs no agent acquire (whose L1 invalidate costs ~1.7 us per wave),
// only a wavefront-scope fence that keeps the compiler from moving the loads above
// the poll.
// A wait that gives up sets a bit of the context's error word and goes on (the
// grid must drain); the word stays set until gsx_sync or gsx_download reports
// it, so no result of a timed-out stage reaches the host as GCMX_OK.
__device__ __forceinline__ void wait_flag(const StageWait& sw, const int* flags, int node) {
	if (sw.budget < 0) {  // test hook: report a timeout without waiting
		atomicOr(sw.err, 1);
		return;
	}
	int polls = 0;
	while (__hip_atomic_load(flags + node, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != sw.epoch) {
		if (++polls > sw.budget) {
			atomicOr(sw.err, 1);
			break;
		}
		__builtin_amdgcn_s_sleep(2);
	}
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Every gradient of the launch is stored (one poll address for all; the sleep
// between polls keeps the polling waves from crowding the counter's updates).
#ifndef GCMX_SX_GPOLL_SLEEP
#define GCMX_SX_GPOLL_SLEEP 2
#endif
__device__ __forceinline__ void wait_gradients(const StageWait& sw) {
	if (sw.budget < 0) {  // test hook: report a timeout without waiting
		atomicOr(sw.err, 2);
		return;
	}
	int polls = 0;
	while ((int)(__hip_atomic_load(sw.gcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - sw.gtarget) < 0) {
		if (++polls > sw.budget) {
			atomicOr(sw.err, 2);
			break;
		}
		__builtin_amdgcn_s_sleep(GCMX_SX_GPOLL_SLEEP);
	}
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// A value another group of the same launch stored: a device-scope atomic (sc1)
// load, never served by this CU's L1 and never hoisted above the wait (the
// kernels' pointers are __restrict__ const, which lets plain loads be treated as
// invariant).
__device__ __forceinline__ double read_ready(const double* p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// TetrahedronInterpolator::hybridInterpolate's (hpp:93-104) gradient term of vertex p
// SHARED: the gradients were stored by other groups of this launch (read_ready).
template <bool SHARED = false>
__device__ __forceinline__ double grad_dot(const double* __restrict__ grad, int p, int k, const double (&d)[3]) {
	const double* gp = grad + (size_t)p * 3 * kG;
	double g[3];
#pragma unroll
	for (int r = 0; r < 3; r++) g[r] = SHARED ? read_ready(gp + r * kG + k) : gp[r * kG + k];
	double dot = g[0] * d[0];
	dot += g[1] * d[1];
	dot += g[2] * d[2];
	return dot;
}

// TetrahedronInterpolator::hybridInterpolate (TetrahedronInterpolator.hpp:93-104)
// of a CELL foot: v = the four vertices' values, dots = each vertex's gradient
// times (q - c_i) (grad_dot's order), lam = q's barycentrics (the host plan's,
// linal::barycentricCoordinates).  The quadratic form (hpp:47-58), the min-max
// limiter of the four values (linal::limiterMinMax), and the linear form (hpp:
// 27-37) when the limiter changed the quadratic value.
__device__ __forceinline__ double tet_linear(const double (&v)[4], const double (&lam)[4]) {
	return lam[0] * v[0] + lam[1] * v[1] + lam[2] * v[2] + lam[3] * v[3];
}
__device__ __forceinline__ double tet_hybrid(const double (&v)[4], const double (&dots)[4], const double (&lam)[4]) {
	double term[4];
#pragma unroll
	for (int i = 0; i < 4; i++) term[i] = v[i] + dots[i] / 2.0;
	const double quadratic = lam[0] * term[0] + lam[1] * term[1] + lam[2] * term[2] + lam[3] * term[3];
	const double mn = std_min(std_min(std_min(v[0], v[1]), v[2]), v[3]);
	const double mx = std_max(std_max(std_max(v[0], v[1]), v[2]), v[3]);
	const double limited = std_min(std_max(quadratic, mn), mx);
	return (quadratic == limited) ? quadratic : tet_linear(v, lam);
}

// interpolateValuesAround for one invariant k (0..5) of node n (node_invariants' body).
// WAIT: the foot's new-invariant reads wait for the border nodes' flags first.
template <bool WAIT = false>
__device__ __forceinline__ double foot_value(int n, int k, int pos, int P, const int4* __restrict__ fv,
                                             const double4* __restrict__ flam,
                                             const int* __restrict__ fmeta, const StageShift& sh,
                                             const double* __restrict__ coords,
                                             const double* __restrict__ w,
                                             const double* __restrict__ grad,
                                             const double* __restrict__ wn, int N,
                                             const StageWait& sw = StageWait{nullptr, nullptr, 0u, 0, nullptr, 0}) {
	double s0 = sh.d[0][0], s1 = sh.d[0][1], s2 = sh.d[0][2];  // shift of invariant k (selects)
#pragma unroll
	for (int kk = 1; kk < 6; kk++)
		if (k == kk) {
			s0 = sh.d[kk][0];
			s1 = sh.d[kk][1];
			s2 = sh.d[kk][2];
		}
	const size_t e = (size_t)k * P + pos;
	const int meta = fmeta[e];
	const int4 f = fv[e];
	const double4 l = flam[e];
	const int kind = meta & 15;
	const int vs[4] = {f.x, f.y, f.z, f.w};
	const double lam[4] = {l.x, l.y, l.z, l.w};
	const double q0 = coords[3 * (size_t)n + 0] + s0, q1 = coords[3 * (size_t)n + 1] + s1,
	             q2 = coords[3 * (size_t)n + 2] + s2;
	double v[4], dots[4], dd[4][3];
	bool waits[4];
	const double* wsrc[4];
	int wnode[4];
#pragma unroll
	for (int i = 0; i < 4; i++) {
		const int p = vs[i];
		const int sl = (meta >> (4 + 4 * i)) & 15;
		const int r = sl < 3 ? sl : sl - 3;
		const int ps = r == 0 ? vs[0] : (r == 1 ? vs[1] : vs[2]);
		const double* src = (kind == GSX_FOOT_CELL) ? w + (size_t)p * kM + k
		                    : (sl < 3)              ? w + (size_t)ps * kM + k
		                                            : wn + (size_t)ps * kM + k;
		// WAIT: a new-invariant value is read after every other load of the foot
		// has been issued (an acquiring poll orders the loads that follow it)
		waits[i] = WAIT && kind == GSX_FOOT_SPACETIME && sl >= 3;
		wsrc[i] = src;
		wnode[i] = ps;
		if (!waits[i]) v[i] = *src;
		dd[i][0] = q0 - coords[3 * (size_t)p + 0];
		dd[i][1] = q1 - coords[3 * (size_t)p + 1];
		dd[i][2] = q2 - coords[3 * (size_t)p + 2];
		if constexpr (!WAIT) dots[i] = grad_dot(grad, p, k, dd[i]);
	}
	if constexpr (WAIT) {
		// only a CELL foot uses the gradients (a SPACETIME foot's terms are unused,
		// hybridInterpolate is not called for it); they come from this launch's
		// gradient groups, so every value above was requested first
		if (kind == GSX_FOOT_CELL && sw.gcount) wait_gradients(sw);
#pragma unroll
		for (int i = 0; i < 4; i++) dots[i] = kind == GSX_FOOT_CELL ? grad_dot<true>(grad, vs[i], k, dd[i]) : 0.0;
#pragma unroll
		for (int i = 0; i < 4; i++)
			if (waits[i]) {
				wait_flag(sw, sw.ready, wnode[i]);
				v[i] = read_ready(wsrc[i]);
			}
	}
	if (kind == GSX_FOOT_CELL) return tet_hybrid(v, dots, lam);
	// interpolateInSpaceTime (common.hpp:102-129): interpolateInOwner's linear form
	if (kind == GSX_FOOT_SPACETIME) return tet_linear(v, lam);
	return 0.0;
}

// All 9 new invariants of node n in every lane of its group (lane c < 6 interpolates
// invariant c, lanes 6, 7 read the exact hits 6, 7; every lane reads 8).
template <bool WAIT = false>
__device__ __forceinline__ void group_invariants(int n, int c, int pos, int P, const int4* __restrict__ fv,
                                                 const double4* __restrict__ flam,
                                                 const int* __restrict__ fmeta, const StageShift& sh,
                                                 const double* __restrict__ coords,
                                                 const double* __restrict__ w,
                                                 const double* __restrict__ grad,
                                                 const double* __restrict__ wn, int N, double (&o)[kM],
                                                 const StageWait& sw = StageWait{nullptr, nullptr, 0u, 0, nullptr, 0}) {
	const double mine = c < 6 ? foot_value<WAIT>(n, c, pos, P, fv, flam, fmeta, sh, coords, w, grad, wn, N, sw)
	                          : w[(size_t)n * kM + c];
	const double w8 = w[(size_t)n * kM + 8];
#pragma unroll
	for (int j = 0; j < kL; j++) o[j] = __shfl(mine, j, kL);
	o[8] = w8;
}

__device__ __forceinline__ double pick9(const double (&o)[kM], int c) {
	double r = o[0];
#pragma unroll
	for (int j = 1; j < kM; j++)
		if (c == j) r = o[j];
	return r;
}

// Row c (and row 8, in every lane) of Mx * in, in mat_vec's order.
__device__ __forceinline__ void rows_mat_vec(const double* __restrict__ Mx, const double (&in)[kM], int c,
                                             double& rc, double& r8) {
	double s = Mx[c * kM + 0] * in[0];
#pragma unroll
	for (int j = 1; j < kM; j++) s += Mx[c * kM + j] * in[j];
	rc = s;
	double t = Mx[8 * kM + 0] * in[0];
#pragma unroll
	for (int j = 1; j < kM; j++) t += Mx[8 * kM + j] * in[j];
	r8 = t;
}

// Rows c and 8 of a 9 x 9 matrix in registers, loaded at the kernel start: a
// matrix entry read where it is used costs one more memory round trip on the
// node's dependent chain (the eight-lane kernels run a few waves per CU, so
// nothing hides it).  rows_mv is rows_mat_vec's arithmetic.
struct Rows2 {
	double rc[kM], r8[kM];
};
__device__ __forceinline__ void load_rows(Rows2& R, const double* __restrict__ Mx, int c) {
#pragma unroll
	for (int j = 0; j < kM; j++) {
		R.rc[j] = Mx[c * kM + j];
		R.r8[j] = Mx[8 * kM + j];
	}
}
__device__ __forceinline__ void rows_mv(const Rows2& R, const double (&in)[kM], double& rc, double& r8) {
	double s = R.rc[0] * in[0];
#pragma unroll
	for (int j = 1; j < kM; j++) s += R.rc[j] * in[j];
	rc = s;
	double t = R.r8[0] * in[0];
#pragma unroll
	for (int j = 1; j < kM; j++) t += R.r8[j] * in[j];
	r8 = t;
}

// finalize() split over the group: lane c writes component c, lane 0 also 8.
// Every store comes after the node's last load: on gfx950 loads and stores share
// vmcnt, so a load issued after a store waits for the store's completion (measured:
// a border launch at 16^3 spent 7 of its 12 us that way).  `wrec`: the border
// kernel's corrected invariants wv, stored node-major when `store_w`.
// R1, Rn: rows c and 8 of U1_s and U_{s+1} (has_next: there is a next stage).
template <bool SC1_W = false>  // wrec is handed off inside the launch: write-through stores
__device__ __forceinline__ void group_finalize(int n, int c, bool store, const double (&wv)[kM],
                                               const Rows2& R1, const Rows2& Rn, bool has_next,
                                               double* __restrict__ un, double* __restrict__ wnext, int N,
                                               double* __restrict__ wrec = nullptr, bool store_w = false) {
	double uc, u8;
	rows_mv(R1, wv, uc, u8);
	double wc = 0.0, w8 = 0.0;
	const bool Unext = has_next;
	if (Unext) {
		double u[kM];
#pragma unroll
		for (int j = 0; j < kL; j++) u[j] = __shfl(uc, j, kL);
		u[8] = u8;
		rows_mv(Rn, u, wc, w8);
	}
	if (store_w && SC1_W) {
		__hip_atomic_store(wrec + (size_t)n * kM + c, pick9(wv, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (c == 0) __hip_atomic_store(wrec + (size_t)n * kM + 8, wv[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	} else if (store_w) {
		wrec[(size_t)n * kM + c] = pick9(wv, c);
		if (c == 0) wrec[(size_t)n * kM + 8] = wv[8];
	}
	if (store) {
		un[(size_t)c * N + n] = uc;
		if (c == 0) un[(size_t)8 * N + n] = u8;
		if (Unext) {
			wnext[(size_t)n * kM + c] = wc;
			if (c == 0) wnext[(size_t)n * kM + 8] = w8;
		}
	}
}

template <bool WAIT>
__device__ __forceinline__ void inner_l8(int gid, const int* __restrict__ nodes, int count,
                                         const int4* __restrict__ fv, const double4* __restrict__ flam,
                                         const int* __restrict__ fmeta, const StageShift& sh,
                                         const double* __restrict__ coords, const double* __restrict__ w,
                                         const double* __restrict__ grad, const double* __restrict__ wn,
                                         const double* __restrict__ U1, const double* __restrict__ Unext,
                                         double* __restrict__ un, double* __restrict__ wnext, int N, int pos0,
                                         int P, const StageWait& sw) {
	const int t = gid / kL, c = gid % kL;
	// whole groups stay active for the shuffles; a group past the list redoes the last node, unstored
	const bool store = t < count;
	const int n = nodes[store ? t : count - 1];
	Rows2 R1, Rn;
	load_rows(R1, U1, c);
	if (Unext) load_rows(Rn, Unext, c);
	double o[kM];
	group_invariants<WAIT>(n, c, pos0 + (store ? t : count - 1), P, fv, flam, fmeta, sh, coords, w, grad, wn,
	                       N, o, sw);
	group_finalize(n, c, store, o, R1, Rn, Unext != nullptr, un, wnext, N);
}

__global__ __launch_bounds__(256) void k_sx_inner_l8(
    const int* __restrict__ nodes, int count, const int4* __restrict__ fv,
    const double4* __restrict__ flam, const int* __restrict__ fmeta, StageShift sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    const double* __restrict__ wn, const double* __restrict__ U1, const double* __restrict__ Unext,
    double* __restrict__ un, double* __restrict__ wnext, int N, int pos0, int P) {
	inner_l8<false>(xcd_gid(), nodes, count, fv, flam, fmeta, sh, coords, w, grad, wn,
	                U1, Unext, un, wnext, N, pos0, P, StageWait{nullptr, nullptr, 0u, 0, nullptr, 0});
}

// The matrix part of calculateOuterWaveCorrection for every border-plan entry t,
// stage s and side (R: Omega = U1 columns 1, 3, 5; L: 0, 2, 4; Model.cpp:81-82):
// B * Omega and its determinant (owc_matrix), md[((t * 3 + s) * 2 + side) * 10].
// Static for a plan and its matrices, so it is evaluated once, not per step.
__global__ __launch_bounds__(256) void k_sx_border_prep(const double* __restrict__ Bm,
                                                        const double* __restrict__ mats, int count,
                                                        double* __restrict__ md) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count * 6) return;
	const int t = i / 6, s = (i / 2) % 3, side = i & 1;
	const double* U1 = mats + 3 * 81 + s * 81;
	const int R[3] = {1, 3, 5}, L[3] = {0, 2, 4};
	double M[3][3];
	const double det = side ? owc_matrix(U1, L, Bm + 27 * (size_t)t, M) : owc_matrix(U1, R, Bm + 27 * (size_t)t, M);
	double* o = md + (size_t)i * 10;
	for (int a = 0; a < 3; a++)
		for (int b = 0; b < 3; b++) o[3 * a + b] = M[a][b];
	o[9] = det;
}

// The stage's corrector record of every border-list position t: the node's plan
// entry ci (-1: not corrected), its condition and outer-wave code, whether each
// side's system is solvable (|det| > minDet of the condition and stage, as
// outer_wave_correction decides), B and the two sides' B * Omega, det -- so the
// border kernel reads them by t, not through node -> entry -> condition.
__global__ __launch_bounds__(256) void k_sx_border_rec(const int* __restrict__ border, int nb,
                                                       const int* __restrict__ corrOf,
                                                       const int* __restrict__ cond,
                                                       const signed char* __restrict__ outer, int count,
                                                       const double* __restrict__ Bm,
                                                       const double* __restrict__ md, int stage,
                                                       const BorderArgs* __restrict__ argp, int4* __restrict__ rec,
                                                       double* __restrict__ recB,
                                                       double* __restrict__ recMd) {
	const BorderArgs& args = *argp;  // static per plan: device memory, not kernel arguments
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= nb) return;
	const int ci = corrOf[border[t]];
	if (ci < 0) {
		rec[t] = make_int4(-1, 0, 0, 0);
		return;
	}
	const int cnd = cond[ci];
	const double* m = md + ((size_t)ci * 3 + stage) * 20;
	const double minValid = args.minDet[cnd][stage];
	const int okR = fabs(m[9]) > minValid, okL = fabs(m[19]) > minValid;
	rec[t] = make_int4(ci, cnd, outer[(size_t)stage * count + ci], okR | (okL << 1) | (args.type[cnd] << 8));
	for (int i = 0; i < 27; i++) recB[(size_t)t * 27 + i] = Bm[27 * (size_t)ci + i];
	for (int i = 0; i < 20; i++) recMd[(size_t)t * 20 + i] = m[i];
}

__device__ __forceinline__ double pick3(const double (&v)[3], int i) {
	return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]);
}

// border_correct (BorderCorrector.hpp:256-265, 118-165) split over the node's group of kL lanes (c = lane in the group,
// h = c / 4, q = c % 4): the U1 and U products by rows; side R in lanes 0-3 and side L
// in lanes 4-7, the matrix part precomputed (k_sx_border_prep, `Md` of this lane's
// side), the residual's three rows over a half's lanes (Brow = row min(q, 2) of B),
// the correction's components q, q + 4 and 8 per lane; the two sides meet through
// one shuffle; both one-sided corrections are always evaluated, so the lanes of a
// wave do not serialise over the nodes' codes.  Every value is produced by
// border_correct's operations in its order.  Returns the node's corrected invariants in every lane of the group.
__device__ __forceinline__ void border_correct_l8(double (&w)[kM], int t, int c, int cnd, int code,
                                                  int okRL, const double (&Brow)[kM],
                                                  const double (&Md)[10], const double (&Sv)[9],
                                                  const Rows2& RU, const Rows2& RU1,
                                                  const double (&cv)[3][3], const double (&b)[3]) {
	const int h = c >> 2, q = c & 3;
	double u[kM], uc, u8;
	rows_mv(RU1, w, uc, u8);  // u = U1 w (mat_vec), rows c and 8 here
#pragma unroll
	for (int j = 0; j < kL; j++) u[j] = __shfl(uc, j, kL);
	u[8] = u8;
	double r[3];
	{  // r_i = b_i - B(i, :) u, row min(q, 2) here
		double x = Brow[0] * u[0];
#pragma unroll
		for (int n = 1; n < kM; n++) x += Brow[n] * u[n];
		const double ri = pick3(b, q < 3 ? q : 2) - x;
#pragma unroll
		for (int i = 0; i < 3; i++) r[i] = __shfl(ri, 4 * h + i, kL);
	}
	const double det = Md[9];
	const double d1 = det3(r[0], Md[1], Md[2], r[1], Md[4], Md[5], r[2], Md[7], Md[8]);
	const double d2 = det3(Md[0], r[0], Md[2], Md[3], r[1], Md[5], Md[6], r[2], Md[8]);
	const double d3 = det3(Md[0], Md[1], r[0], Md[3], Md[4], r[1], Md[6], Md[7], r[2]);
	const double alpha[3] = {d1 / det, d2 / det, d3 / det};
	// cv[r][j] = U1(row, c0 + 2 j) for rows q, q + 4, 8, with c0 = 1 - h: this
	// side's columns (R: 1, 3, 5; L: 0, 2, 4)
	auto value = [&](int r) {
		double x = cv[r][0] * alpha[0];
		x += cv[r][1] * alpha[1];
		x += cv[r][2] * alpha[2];
		return x;
	};
	const double vq = value(0), vq4 = value(1), v8 = value(2);
	// this side's value of the own component c, the other side's from the partner c ^ 4
	const double mine = h ? vq4 : vq;
	const double other = __shfl_xor(h ? vq : vq4, 4, kL);
	const double other8 = __shfl_xor(v8, 4, kL);
	const double vrc = h ? other : mine, vlc = h ? mine : other;
	const double vr8 = h ? other8 : v8, vl8 = h ? v8 : other8;
	const bool okR = okRL & 1, okL = (okRL >> 1) & 1;
	bool plain = false;
	if (code == 1 || code == 2) {
		if (code == 1 ? okR : okL) {
			uc += code == 1 ? vrc : vlc;
			u8 += code == 1 ? vr8 : vl8;
		} else {
			plain = true;
		}
	} else {
		if (okR && okL) {
			uc += (vrc + vlc) / 2;
			u8 += (vr8 + vl8) / 2;
		} else {
			plain = true;
		}
	}
	double up[kM];  // the plain correction: per node, so the whole group takes it
#pragma unroll
	for (int j = 0; j < kM; j++) up[j] = u[j];
	if (plain) plain_correction(up, okRL >> 8, Sv, b);
#pragma unroll
	for (int j = 0; j < kL; j++) {
		const double sj = __shfl(uc, j, kL);
		u[j] = plain ? up[j] : sj;
	}
	u[8] = plain ? up[8] : u8;
	double wc, w8;  // w = U u (mat_vec), rows c and 8 here
	rows_mv(RU, u, wc, w8);
#pragma unroll
	for (int j = 0; j < kL; j++) w[j] = __shfl(wc, j, kL);
	w[8] = w8;
}

// SIGNAL: publish each node's flag once its wn is stored (k_sx_stage_l8).
template <bool SIGNAL>
__device__ __forceinline__ void border_l8(
    int gid, const int* __restrict__ nodes, int count, const int4* __restrict__ fv,
    const double4* __restrict__ flam, const int* __restrict__ fmeta, const StageShift& sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    double* __restrict__ wn, const char* __restrict__ deferred, const BorderDevArgs& bp,
    const BorderArgs* __restrict__ argp, const double* __restrict__ U, const double* __restrict__ U1,
    const double* __restrict__ Unext, double* __restrict__ un, double* __restrict__ wnext, int stage, int N,
    int pos0, int P, const StageWait& sw) {
	const BorderArgs& args = *argp;  // static per plan: device memory, not kernel arguments
#ifndef GCMX_SX_L8_STAGE  // tuning: stage U / U1 / U_next in LDS (1) or read them through the caches (0)
#define GCMX_SX_L8_STAGE 0
#endif
#if GCMX_SX_L8_STAGE
	__shared__ SharedMats<3> sm;
	stage_mats<3>(sm, {U, U1, Unext});
	const double* Us = sm.m[0];
	const double* U1s = sm.m[1];
	const double* Uns = Unext ? sm.m[2] : nullptr;
#else
	const double* Us = U;
	const double* U1s = U1;
	const double* Uns = Unext;
#endif
	const int t = gid / kL, c = gid % kL;
	const bool store = t < count;
	const int n = nodes[store ? t : count - 1];
	// the node's corrector data first: its loads overlap the feet's gathers
	// the node's corrector record first (by list position: no dependent loads), so
	// its loads overlap the feet's gathers
	const int tr = store ? t : count - 1;
	const int4 rc = bp.cond ? bp.rec[tr] : make_int4(-1, 0, 0, 0);
	const int ci = rc.x, cnd = rc.y, code = rc.z;
	double Brow[kM], Md[10], cv[3][3], Sv[9], bv[3] = {0.0, 0.0, 0.0};
	Rows2 RU, RU1, Rn;  // every matrix entry the node needs, loaded up front
	load_rows(RU1, U1s, c);
	if (Uns) load_rows(Rn, Uns, c);
	const bool fin = store && !deferred[n];
	if (ci >= 0) {
		const int q = c & 3, h = c >> 2;
		const double* Bi = bp.recB + 27 * (size_t)tr + kM * (q < 3 ? q : 2);
#pragma unroll
		for (int i = 0; i < kM; i++) Brow[i] = Bi[i];
		const double* m = bp.recMd + (size_t)tr * 20 + h * 10;
#pragma unroll
		for (int i = 0; i < 10; i++) Md[i] = m[i];
		load_rows(RU, Us, c);
		const double* Si = bp.S + 9 * (size_t)ci;
#pragma unroll
		for (int i = 0; i < 9; i++) Sv[i] = Si[i];
#pragma unroll
		for (int i = 0; i < 3; i++) bv[i] = args.b[3 * cnd + i];  // the step's b(t) of the condition
		const int rows[3] = {q, q + 4, 8};
#pragma unroll
		for (int r = 0; r < 3; r++)
#pragma unroll
			for (int j = 0; j < 3; j++) cv[r][j] = U1s[rows[r] * kM + (1 - h) + 2 * j];
	}
	double o[kM];
	// in the one-launch stage the feet wait for their cells' gradients (never for wn:
	// the plan check keeps new-invariant reads out of border feet)
	group_invariants<SIGNAL>(n, c, pos0 + tr, P, fv, flam, fmeta, sh, coords, w, grad, wn, N, o, sw);
#ifndef GCMX_SX_DIAG_NOCORR  // tuning builds only: time the kernel without the correctors
	if (ci >= 0) border_correct_l8(o, ci, c, cnd, code, rc.w, Brow, Md, Sv, RU, RU1, cv, bv);
#endif
	// wn (node-major, like wnext) is stored with the finalisation's stores, after every load
	group_finalize<SIGNAL>(n, c, fin, o, RU1, Rn, Uns != nullptr, un, wnext, N, wn, store);
	if constexpr (SIGNAL) {
		// the group's eight lanes are one wave's: drain their sc1 wn stores, then the flag
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		if (c == 0 && store)
			__hip_atomic_store(sw.ready + n, sw.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}

__global__ __launch_bounds__(256) void k_sx_border_l8(
    const int* __restrict__ nodes, int count, const int4* __restrict__ fv,
    const double4* __restrict__ flam, const int* __restrict__ fmeta, StageShift sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    double* __restrict__ wn, const char* __restrict__ deferred, BorderDevArgs bp, const BorderArgs* __restrict__ argp,
    const double* __restrict__ U, const double* __restrict__ U1, const double* __restrict__ Unext,
    double* __restrict__ un, double* __restrict__ wnext, int stage, int N, int pos0, int P) {
	border_l8<false>(xcd_gid(), nodes, count, fv, flam, fmeta, sh, coords, w, grad, wn,
	                 deferred, bp, argp, U, U1, Unext, un, wnext, stage, N, pos0, P, StageWait{nullptr, nullptr, 0u, 0, nullptr, 0});
}

// One launch for a whole stage of one body (gsx_stage, nothing between its
// border and inner halves): blocks [0, ngBlk) run k_sx_gradient_l8's groups,
// [ngBlk, ngBlk + nbBlk) k_sx_border_l8's over the border list, the rest
// k_sx_inner_l8's over the inner list, side by side.  A CELL foot waits until
// every gradient block has finished.
// An inner foot interpolating in space-time with border nodes' NEW invariants
// (interpolateInOwner; engine/simplex/Engine.cpp:119-135 orders the border
// stage first) waits for exactly those nodes' flags.  Every wait is on blocks
// with LOWER ids: inner groups wait on border and gradient blocks, border groups
// (their CELL feet, mode 2) only on gradient blocks, gradient blocks never wait.
// No dispatch-order assumption: a block's work index is not blockIdx.x but a
// TICKET it takes from a per-context counter when it starts (one atomic per
// block).  Tickets are handed out in the order blocks start running, so the
// lower-index work a block waits for belongs to blocks that already started --
// resident or finished -- whatever order the hardware dispatches workgroups in,
// and every wait can end.  Every wait stays bounded (StageWait::budget) as a
// backstop; the grid is capped at kFuseMaxBlocks (4096) blocks for speed only.
__global__ __launch_bounds__(256) void k_sx_stage_l8(
    const int* __restrict__ border, int nBorder, const int* __restrict__ inner, int nInner, int nbBlk,
    const int4* __restrict__ fv, const double4* __restrict__ flam, const int* __restrict__ fmeta, StageShift sh,
    const double* __restrict__ coords, const double* __restrict__ w, const double* __restrict__ grad,
    double* __restrict__ wn, const char* __restrict__ deferred, BorderDevArgs bp, const BorderArgs* __restrict__ argp,
    const double* __restrict__ U, const double* __restrict__ U1, const double* __restrict__ Unext,
    double* __restrict__ un, double* __restrict__ wnext, int stage, int N, StageWait sw, int ngBlk,
    double* __restrict__ gradw, const int* __restrict__ gOff, const int* __restrict__ gNb,
    const double* __restrict__ gW, const double* __restrict__ gM, const double* __restrict__ gDet) {
	const int P = nBorder + nInner;
	__shared__ unsigned ticket;
	if (threadIdx.x == 0) ticket = __hip_atomic_fetch_add(sw.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__syncthreads();
	const int b = (int)(ticket - sw.tbase);  // work index, in start order
	if (b < ngBlk)
		gradient_l8<true>(b * blockDim.x + threadIdx.x, w, gradw, gOff, gNb, coords, gW, gM, gDet, N, sw.gcount);
	else if (b < ngBlk + nbBlk)
		border_l8<true>((b - ngBlk) * blockDim.x + threadIdx.x, border, nBorder, fv, flam, fmeta, sh, coords, w, grad,
		                wn, deferred, bp, argp, U, U1, Unext, un, wnext, stage, N, 0, P, sw);
	else
		inner_l8<true>((b - ngBlk - nbBlk) * blockDim.x + threadIdx.x, inner, nInner, fv, flam, fmeta, sh, coords,
		               w, grad, wn, U1, Unext, un, wnext, N, nBorder, P, sw);
}

// The step's border values b(t) into device memory (gsx_set_border_values).
struct BorderValues {
	double b[3 * GSX_MAX_BORDER_CONDITIONS];
};
__global__ __launch_bounds__(64) void k_sx_set_border_values(double* __restrict__ dst, BorderValues v,
                                                             int n) {
	for (int i = threadIdx.x; i < n; i += 64) dst[i] = v.b[i];
}

// BorderCorrectorInPdeVectors::applyPlainCorrection (BorderCorrector.hpp:167-178) on
// the current layer.
__global__ __launch_bounds__(64) void k_sx_plain(const int* __restrict__ nodes,
                                                  const int* __restrict__ cond,
                                                  const double* __restrict__ Sm, double* u_,
                                                  int count, int N, const BorderArgs* __restrict__ argp) {
	const BorderArgs& args = *argp;  // static per plan: device memory, not kernel arguments
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= count) return;
	const int n = nodes[t], c = cond[t];
	const double b[3] = {args.b[3 * c], args.b[3 * c + 1], args.b[3 * c + 2]};
	double u[kM];
	for (int k = 0; k < kM; k++) u[k] = u_[k * N + n];
	plain_correction(u, args.type[c], Sm + 9 * (size_t)t, b);
	for (int k = 0; k < kM; k++) u_[k * N + n] = u[k];
}

// The plain border corrections (as k_sx_plain) of the plan's nodes fused with the
// first stage's beforeStage (w = U_0 u, as k_sx_transform<true>) of every node:
// both act on one node's own vector, so one pass does the step's start.
__global__ __launch_bounds__(256) void k_sx_begin(double* u_, double* __restrict__ w,
                                                  const double* __restrict__ U0,
                                                  const int2* __restrict__ nodeRec,
                                                  const double* __restrict__ Sm, int N, const BorderArgs* __restrict__ argp) {
	const BorderArgs& args = *argp;  // static per plan: device memory, not kernel arguments
	const int n = xcd_gid();
	if (n >= N) return;
	double u[kM];
#pragma unroll
	for (int k = 0; k < kM; k++) u[k] = u_[k * N + n];
	const int2 rc = nodeRec ? nodeRec[n] : make_int2(-1, 0);  // (entry, condition)
	const int t = rc.x;
	if (t >= 0) {
		const int c = rc.y;
		const double b[3] = {args.b[3 * c], args.b[3 * c + 1], args.b[3 * c + 2]};
		plain_correction(u, args.type[c], Sm + 9 * (size_t)t, b);
		for (int k = 0; k < kM; k++) u_[k * N + n] = u[k];
	}
	double wv[kM];
	mat_vec(U0, u, wv);
#pragma unroll
	for (int k = 0; k < kM; k++) w[(size_t)n * kM + k] = wv[k];
}

// ContactCorrectorInRiemannInvariants::applyInGlobalBasis (ContactCorrector.hpp:333-348):
// matchInnersAndOuters (zeroing decided on the host), invariants -> PDE (U1),
// ContactCorrectorInPdeVectors::applyInGlobalBasis (:150-247), PDE -> invariants (U).
__global__ __launch_bounds__(64) void k_sx_contact(
    const int* __restrict__ na, const int* __restrict__ nb, const double* __restrict__ normal,
    const double* __restrict__ Sm, const signed char* __restrict__ codeA,
    const signed char* __restrict__ codeB, const double* __restrict__ UA_,
    const double* __restrict__ U1A_, const double* __restrict__ UB_, const double* __restrict__ U1B_,
    double* wnA, double* wnB, int NA, int NB, int count, int stage, double min1, double min2,
    const double* __restrict__ UnextA_, const double* __restrict__ UnextB_, double* unA, double* unB,
    double* wnextA, double* wnextB) {
	__shared__ SharedMats<6> sm;
	stage_mats<6>(sm, {UA_, U1A_, UB_, U1B_, UnextA_, UnextB_});
	const double* UA = sm.m[0];
	const double* U1A = sm.m[1];
	const double* UB = sm.m[2];
	const double* U1B = sm.m[3];
	const double* UnextA = UnextA_ ? sm.m[4] : nullptr;
	const double* UnextB = UnextB_ ? sm.m[5] : nullptr;
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= count) return;
	const int a = na[t], b = nb[t];
	const int ca = codeA[(size_t)stage * count + t], cb = codeB[(size_t)stage * count + t];
	const int R[3] = {1, 3, 5}, L[3] = {0, 2, 4};  // Model.cpp:81-82
	double wA[kM], wB[kM], uA[kM], uB[kM];
	for (int k = 0; k < kM; k++) {
		wA[k] = wnA[(size_t)a * kM + k];
		wB[k] = wnB[(size_t)b * kM + k];
	}
	auto zero = [&](double (&w)[kM], int code) {
		if (!(code & 4)) return;
		if (code & 1) w[1] = w[3] = w[5] = 0;
		if (code & 2) w[0] = w[2] = w[4] = 0;
	};
	zero(wA, ca);
	zero(wB, cb);
	mat_vec(U1A, wA, uA);
	mat_vec(U1B, wB, uB);
	const double n[3] = {normal[3 * t], normal[3 * t + 1], normal[3 * t + 2]};
	double S[3][3];
	for (int i = 0; i < 9; i++) S[i / 3][i % 3] = Sm[9 * (size_t)t + i];
	double B1[3][kM], B2[3][kM];
	gsx::fixedVelocityGlobal(B1);
	gsx::fixedForceGlobal(n, B2);
	const int oa = ca & 3, ob = cb & 3;
	const int sa = oa == 0 ? 0 : oa == 3 ? 6 : 3, sb = ob == 0 ? 0 : ob == 3 ? 6 : 3;
	if (sa == 3 && sb == 3) {
		const auto c = gsx::contactCorrection(uA, U1A, oa == 1 ? R : L, uB, U1B, ob == 1 ? R : L, B1,
		                                      B2, min1, min2);
		if (c.ok) {
			for (int k = 0; k < kM; k++) {
				uA[k] += c.valueA[k];
				uB[k] += c.valueB[k];
			}
		} else {
			gsx::plainContactAverage(uA, uB, S);
		}
	} else if (sa == 6 && sb == 0) {
		double v[kM];
		if (gsx::doubleBorderCorrection(uA, U1A, uB, B1, B2, min1, v)) {
			for (int k = 0; k < kM; k++) uA[k] += v[k];
		} else {
			gsx::plainContactOneSided(uA, uB, S);
		}
	} else if (sb == 6 && sa == 0) {
		double v[kM];
		if (gsx::doubleBorderCorrection(uB, U1B, uA, B1, B2, min1, v)) {
			for (int k = 0; k < kM; k++) uB[k] += v[k];
		} else {
			gsx::plainContactOneSided(uB, uA, S);
		}
	} else {
		const auto c1 = gsx::contactCorrection(uA, U1A, R, uB, U1B, L, B1, B2, min1, min2);
		const auto c2 = gsx::contactCorrection(uA, U1A, L, uB, U1B, R, B1, B2, min1, min2);
		if (c1.ok && c2.ok) {
			for (int k = 0; k < kM; k++) {
				uA[k] += (c1.valueA[k] + c2.valueA[k]) / 2;
				uB[k] += (c1.valueB[k] + c2.valueB[k]) / 2;
			}
		} else {
			gsx::plainContactAverage(uA, uB, S);
		}
	}
	mat_vec(UA, uA, wA);
	mat_vec(UB, uB, wB);
	for (int k = 0; k < kM; k++) {
		wnA[(size_t)a * kM + k] = wA[k];
		wnB[(size_t)b * kM + k] = wB[k];
	}
	finalize(a, wA, U1A, UnextA, unA, wnextA, NA);
	finalize(b, wB, U1B, UnextB, unB, wnextB, NB);
}

// ContactCorrectorInPdeVectors::applyPlainCorrection (ContactCorrector.hpp:249-262)
// on the current layers.
__global__ __launch_bounds__(256) void k_sx_contact_plain(const int* __restrict__ na,
                                                          const int* __restrict__ nb,
                                                          const double* __restrict__ Sm,
                                                          double* uA_, double* uB_, int NA, int NB,
                                                          int count) {
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= count) return;
	const int a = na[t], b = nb[t];
	double uA[kM], uB[kM], S[3][3];
	for (int k = 0; k < kM; k++) {
		uA[k] = uA_[k * NA + a];
		uB[k] = uB_[k * NB + b];
	}
	for (int i = 0; i < 9; i++) S[i / 3][i % 3] = Sm[9 * (size_t)t + i];
	gsx::plainContactAverage(uA, uB, S);
	for (int k = 0; k < kM; k++) {
		uA_[k * NA + a] = uA[k];
		uB_[k * NB + b] = uB[k];
	}
}

gcmx_status check(gsx_ctx* c) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null simplex context");
	SX_TRY(hipSetDevice(c->device));
	return GCMX_OK;
}

template <class T>
gcmx_status upload(T** dst, const T* src, size_t n) {
	if (*dst) SX_TRY(hipFree(*dst));
	*dst = nullptr;
	if (n == 0) return GCMX_OK;
	SX_TRY(hipMalloc(dst, n * sizeof(T)));
	SX_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
	return GCMX_OK;
}

// The corrector matrices of the current border plan and matrices (k_sx_border_prep)
// and every set stage's records (k_sx_border_rec), enqueued on the context stream
// whenever one of matrices, border plan or a stage plan is (re)set.
gcmx_status prep_border(gsx_ctx* c) {
	BorderDev& bd = c->bd;
	if (!c->matsSet || !bd.set || bd.n == 0) return GCMX_OK;
	if (!bd.md) SX_TRY(hipMalloc(&bd.md, (size_t)bd.n * 60 * sizeof(double)));
	SX_LAUNCH(c, k_sx_border_prep, dim3(((size_t)bd.n * 6 + 255) / 256), dim3(256), 0, c->stream,
	                   bd.B, c->mats, bd.n, bd.md);
	SX_TRY(hipGetLastError());
	for (int s = 0; s < 3; s++) {
		StageDev& st = c->st[s];
		if (!st.set || st.nBorder == 0) continue;
		if (!st.rec) {
			SX_TRY(hipMalloc(&st.rec, (size_t)st.nBorder * sizeof(int4)));
			SX_TRY(hipMalloc(&st.recB, (size_t)st.nBorder * 27 * sizeof(double)));
			SX_TRY(hipMalloc(&st.recMd, (size_t)st.nBorder * 20 * sizeof(double)));
		}
		SX_LAUNCH(c, k_sx_border_rec, dim3((st.nBorder + 255) / 256), dim3(256), 0, c->stream,
		                   st.border, st.nBorder, c->corrOf, bd.cond, bd.outer, bd.n, bd.B, bd.md, s,
		                   bd.argsDev, st.rec, st.recB, st.recMd);
		SX_TRY(hipGetLastError());
	}
	return GCMX_OK;
}

}  // namespace

namespace {
// Body b's stream work so far precedes the launch on a's stream, and the launch
// precedes b's later work.
template <class Launch>
gcmx_status onBothStreams(gsx_contact* c, Launch launch) {
	SX_TRY(hipEventRecord(c->evB, c->b->stream));
	SX_TRY(hipStreamWaitEvent(c->a->stream, c->evB, 0));
	launch();
	SX_TRY(hipGetLastError());
	SX_TRY(hipEventRecord(c->evA, c->a->stream));
	SX_TRY(hipStreamWaitEvent(c->b->stream, c->evA, 0));
	return GCMX_OK;
}
}  // namespace

extern "C" {

gcmx_status gsx_create(int device, int n_nodes, const double* coords, gsx_ctx** out) {
	if (!out || n_nodes <= 0 || !coords) return fail(GCMX_ERR_INVALID_ARG, "bad gsx_create arguments");
	*out = nullptr;
	int nd = 0;
	SX_TRY(hipGetDeviceCount(&nd));
	if (device < 0 || device >= nd) return fail(GCMX_ERR_INVALID_ARG, "no such device");
	gsx_ctx* c = new gsx_ctx();
	c->device = device;
	c->N = n_nodes;
	SX_TRY(hipSetDevice(device));
	SX_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
	const size_t N = (size_t)n_nodes;
	c->hostCoords.assign(coords, coords + 3 * N);
	gcmx_status s = upload(&c->coords, coords, 3 * N);  // node-major [n][3]
	if (s) { gsx_destroy(c); return s; }
	// The per-step node arrays live in one allocation (2 MiB-aligned pieces of one
	// range): the node kernels of a small mesh touch all of them every stage, and
	// a few large pages keep their address translations resident.
	double** bufs[6] = {&c->u, &c->un, &c->w, &c->wn, &c->grad, &c->wnext};
	const size_t sizes[6] = {kM * N, kM * N, kM * N, kM * N, 3 * 6 * N, kM * N};
	size_t total = 0;
	for (int i = 0; i < 6; i++) total += (sizes[i] + 31) / 32 * 32;  // 256-byte aligned pieces
	if (hipMalloc(&c->arena, total * sizeof(double)) != hipSuccess ||
	    hipMemset(c->arena, 0, total * sizeof(double)) != hipSuccess) {
		gsx_destroy(c);
		return fail(GCMX_ERR_OOM, "simplex layer allocation failed");
	}
	for (size_t i = 0, o = 0; i < 6; o += (sizes[i] + 31) / 32 * 32, i++) *bufs[i] = c->arena + o;
	c->hostDeferred.assign(N, 0);
	if ((s = upload(&c->deferred, c->hostDeferred.data(), N))) {
		gsx_destroy(c);
		return s;
	}
	if (hipMalloc(&c->bvals, 3 * GSX_MAX_BORDER_CONDITIONS * sizeof(double)) != hipSuccess ||
	    hipMemset(c->bvals, 0, 3 * GSX_MAX_BORDER_CONDITIONS * sizeof(double)) != hipSuccess) {
		gsx_destroy(c);
		return fail(GCMX_ERR_OOM, "simplex border-value allocation failed");
	}
	// [0, N) border flags, [N] finished-gradient-block counter, [N + 1] error word,
	// [N + 2] work-ticket counter of k_sx_stage_l8
	if (hipMalloc(&c->ready, (N + 3) * sizeof(int)) != hipSuccess ||
	    hipMemset(c->ready, 0, (N + 3) * sizeof(int)) != hipSuccess) {
		gsx_destroy(c);
		return fail(GCMX_ERR_OOM, "simplex flag allocation failed");
	}
	*out = c;
	return GCMX_OK;
}

void gsx_destroy(gsx_ctx* c) {
	if (!c) return;
	(void)hipSetDevice(c->device);
	if (c->stream) (void)hipStreamSynchronize(c->stream);
	c->graphs.reset();
	if (c->bvals) (void)hipFree(c->bvals);
	if (c->ready) (void)hipFree(c->ready);
	void* ptrs[] = {c->coords, c->arena, c->corrOf, c->deferred,
	                c->mats, c->gOff, c->gNb,
	                c->gRows, c->gW, c->gM, c->gDet};
	for (void* p : ptrs)
		if (p) (void)hipFree(p);
	void* bptrs[] = {c->bd.nodes, c->bd.cond, c->bd.B, c->bd.S, c->bd.outer, c->bd.md, c->bd.nodeRec,
	                 c->bd.argsDev};
	for (void* p : bptrs)
		if (p) (void)hipFree(p);
	for (auto& st : c->st) {
		if (st.fv) (void)hipFree(st.fv);
		if (st.flam) (void)hipFree(st.flam);
		if (st.fmeta) (void)hipFree(st.fmeta);
		if (st.border) (void)hipFree(st.border);
		if (st.inner) (void)hipFree(st.inner);
		if (st.rec) (void)hipFree(st.rec);
		if (st.recB) (void)hipFree(st.recB);
		if (st.recMd) (void)hipFree(st.recMd);
	}
	if (c->stream) (void)hipStreamDestroy(c->stream);
	delete c;
}

gcmx_status gsx_set_matrices(gsx_ctx* c, const double* U, const double* U1) {
	gcmx_status s = check(c);
	if (s) return s;
	c->planGen++;  // captured step graphs point into what this call replaces
	if (!U || !U1) return fail(GCMX_ERR_INVALID_ARG, "null matrices");
	std::vector<double> m(2 * 3 * 81);
	std::memcpy(m.data(), U, 3 * 81 * sizeof(double));
	std::memcpy(m.data() + 3 * 81, U1, 3 * 81 * sizeof(double));
	SX_TRY(hipStreamSynchronize(c->stream));
	s = upload(&c->mats, m.data(), m.size());
	if (s) return s;
	c->matsSet = true;
	c->wStage = -1;
	return prep_border(c);
}

gcmx_status gsx_set_gradient_plan(gsx_ctx* c, const int* off, const int* nbs, const double* rows,
                                  const double* wts, const double* M, const double* det) {
	gcmx_status s = check(c);
	if (s) return s;
	c->planGen++;  // captured step graphs point into what this call replaces
	if (!off || !nbs || !rows || !wts || !M || !det)
		return fail(GCMX_ERR_INVALID_ARG, "null gradient plan");
	const int N = c->N, E = off[N];
	if (off[0] != 0 || E < 0) return fail(GCMX_ERR_INVALID_ARG, "bad gradient offsets");
	for (int n = 0; n < N; n++) {
		const int K = off[n + 1] - off[n];
		if (K < 1 || K > kMaxNb) return fail(GCMX_ERR_INVALID_ARG, "1..20 neighbours per node expected");
		if (!(det[n] != 0)) return fail(GCMX_ERR_INVALID_ARG, "singular gradient system");
		for (int e = off[n]; e < off[n + 1]; e++) {
			if (nbs[e] < 0 || nbs[e] >= N) return fail(GCMX_ERR_INVALID_ARG, "neighbour out of range");
			// the device recomputes the LSQ row from the coordinates
			for (int r = 0; r < 3; r++)
				if (!(c->hostCoords[3 * (size_t)nbs[e] + r] - c->hostCoords[3 * (size_t)n + r] ==
				      rows[3 * (size_t)e + r]))
					return fail(GCMX_ERR_INVALID_ARG, "gradient row is not coords[nb] - coords[n]");
		}
	}
	SX_TRY(hipStreamSynchronize(c->stream));
	if ((s = upload(&c->gOff, off, (size_t)N + 1)) || (s = upload(&c->gNb, nbs, (size_t)E)) ||
	    (s = upload(&c->gW, wts, (size_t)E)) || (s = upload(&c->gM, M, 9 * (size_t)N)) ||
	    (s = upload(&c->gDet, det, (size_t)N)))
		return s;
	c->gradSet = true;
	return GCMX_OK;
}

gcmx_status gsx_set_stage_plan(gsx_ctx* c, int stage, const gsx_foot* feet, const double* shift,
                               int nb, const int* border, int ni, const int* inner) {
	gcmx_status s = check(c);
	if (s) return s;
	c->planGen++;  // captured step graphs point into what this call replaces
	if (stage < 0 || stage > 2 || !feet || !shift || nb < 0 || ni < 0 || (nb && !border) ||
	    (ni && !inner))
		return fail(GCMX_ERR_INVALID_ARG, "bad stage plan");
	const int N = c->N;
	for (int i = 0; i < nb; i++)
		if (border[i] < 0 || border[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "node out of range");
	for (int i = 0; i < ni; i++)
		if (inner[i] < 0 || inner[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "node out of range");
	// feet stored by list position (border list, then inner list), [k][pos]: the
	// node kernels read them by the thread's position, not through the node id
	const int P = nb + ni;
	std::vector<int4> fv((size_t)P * 6);
	std::vector<double4> flam((size_t)P * 6);
	std::vector<int> fmeta((size_t)P * 6);
	for (int pos = 0; pos < P; pos++)
		for (int k = 0; k < 6; k++) {
			const int n = pos < nb ? border[pos] : inner[pos - nb];
			const gsx_foot& f = feet[(size_t)n * 6 + k];
			const int nv = f.kind == GSX_FOOT_CELL ? 4 : f.kind == GSX_FOOT_SPACETIME ? 3 : 0;
			if (f.kind < 0 || f.kind > 3) return fail(GCMX_ERR_INVALID_ARG, "bad foot kind");
			for (int i = 0; i < nv; i++)
				if (f.v[i] < 0 || f.v[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "foot vertex out of range");
			int meta = f.kind;
			if (f.kind == GSX_FOOT_SPACETIME)
				for (int i = 0; i < 4; i++) {
					if (f.slot[i] < 0 || f.slot[i] > 5) return fail(GCMX_ERR_INVALID_ARG, "bad slot");
					meta |= f.slot[i] << (4 + 4 * i);
				}
			if (f.kind == GSX_FOOT_CELL)
				for (int r = 0; r < 3; r++)
					if (!(c->hostCoords[3 * (size_t)n + r] + shift[k * 3 + r] == f.q[r]))
						return fail(GCMX_ERR_INVALID_ARG, "foot point is not node + shift");
			const size_t e = (size_t)k * P + pos;
			fv[e] = make_int4(nv > 0 ? f.v[0] : 0, nv > 1 ? f.v[1] : 0, nv > 2 ? f.v[2] : 0,
			                  nv > 3 ? f.v[3] : 0);
			flam[e] = make_double4(f.lam[0], f.lam[1], f.lam[2], f.lam[3]);
			fmeta[e] = meta;
		}
	// Inner nodes whose feet read border nodes' new invariants (wn) go to the END
	// of the inner list (stable): in the one-launch stage they are the only
	// groups that wait, so the independent ones fill the low block ids, finish
	// and retire while the border groups run.  Every node is computed on its own,
	// so the order changes no result.
	std::vector<int> innerOrd(inner, inner + ni);
	{
		auto readsWn = [&](int pos) {
			for (int k = 0; k < 6; k++) {
				const size_t e = (size_t)k * P + pos;
				if ((fmeta[e] & 15) != GSX_FOOT_SPACETIME) continue;
				for (int i = 0; i < 4; i++)
					if (((fmeta[e] >> (4 + 4 * i)) & 15) >= 3) return true;
			}
			return false;
		};
		std::vector<int> perm;  // new inner position -> old inner position
		perm.reserve(ni);
		for (int i = 0; i < ni; i++)
			if (!readsWn(nb + i)) perm.push_back(i);
		for (int i = 0; i < ni; i++)
			if (readsWn(nb + i)) perm.push_back(i);
		std::vector<int4> fv2(fv);
		std::vector<double4> flam2(flam);
		std::vector<int> fmeta2(fmeta);
		for (int j = 0; j < ni; j++) {
			innerOrd[j] = inner[perm[j]];
			for (int k = 0; k < 6; k++) {
				const size_t dst = (size_t)k * P + nb + j, src = (size_t)k * P + nb + perm[j];
				fv2[dst] = fv[src];
				flam2[dst] = flam[src];
				fmeta2[dst] = fmeta[src];
			}
		}
		fv.swap(fv2);
		flam.swap(flam2);
		fmeta.swap(fmeta2);
	}
	// one-launch stage (k_sx_stage_l8): every wn read of an inner foot must name a
	// node of the border list (its flag is set in the same launch), and no border
	// foot may read wn (border groups never wait)
	bool fusable = true;
	int waitFeet = 0;  // inner feet that read border nodes' new invariants (they wait in one launch)
	{
		std::vector<char> inBorder(N, 0);
		for (int i = 0; i < nb; i++) inBorder[border[i]] = 1;
		for (int pos = 0; pos < P; pos++)
			for (int k = 0; k < 6; k++) {
				const size_t e = (size_t)k * P + pos;
				if ((fmeta[e] & 15) != GSX_FOOT_SPACETIME) continue;
				const int vs[4] = {fv[e].x, fv[e].y, fv[e].z, fv[e].w};
				bool reads_wn = false;
				for (int i = 0; i < 4; i++) {
					const int sl = (fmeta[e] >> (4 + 4 * i)) & 15;
					if (sl < 3) continue;
					reads_wn = true;
					if (pos < nb || !inBorder[vs[sl - 3]]) fusable = false;
				}
				if (reads_wn && pos >= nb) waitFeet++;
			}
	}
	SX_TRY(hipStreamSynchronize(c->stream));
	StageDev& st = c->st[stage];
	if ((s = upload(&st.fv, fv.data(), fv.size())) || (s = upload(&st.flam, flam.data(), flam.size())) ||
	    (s = upload(&st.fmeta, fmeta.data(), fmeta.size())) ||
	    (s = upload(&st.border, border, (size_t)nb)) || (s = upload(&st.inner, innerOrd.data(), (size_t)ni)))
		return s;
	for (int k = 0; k < 6; k++)
		for (int r = 0; r < 3; r++) st.shift.d[k][r] = shift[k * 3 + r];
	if (st.rec && st.nBorder != nb) {  // the records are sized by the border list
		SX_TRY(hipFree(st.rec));
		SX_TRY(hipFree(st.recB));
		SX_TRY(hipFree(st.recMd));
		st.rec = nullptr;
		st.recB = st.recMd = nullptr;
	}
	st.nBorder = nb;
	st.nInner = ni;
	st.fusable = fusable;
	st.waitFeet = waitFeet;
	st.set = true;
	return prep_border(c);
}

}  // extern "C"

// After a stream synchronisation: the error word of the one-launch stages (a
// device wait that gave up), reported once and cleared.
static gcmx_status report_wait_error(gsx_ctx* c) {
	if (!c->ready) return GCMX_OK;
	int err = 0;
	SX_TRY(hipMemcpy(&err, c->ready + (size_t)c->N + 1, sizeof(int), hipMemcpyDeviceToHost));
	if (!err) return GCMX_OK;
	SX_TRY(hipMemset(c->ready + (size_t)c->N + 1, 0, sizeof(int)));
	return fail(GCMX_ERR_STATE, err & 2 ? "one-launch simplex stage: a gradient wait timed out (results invalid)"
	                                    : "one-launch simplex stage: a border-node wait timed out (results invalid)");
}

extern "C" {

gcmx_status gsx_upload(gsx_ctx* c, const double* aos) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!aos) return fail(GCMX_ERR_INVALID_ARG, "null layer");
	const size_t N = (size_t)c->N;
	std::vector<double> soa(kM * N);
	for (size_t n = 0; n < N; n++)
		for (int k = 0; k < kM; k++) soa[k * N + n] = aos[kM * n + k];
	SX_TRY(hipStreamSynchronize(c->stream));
	SX_TRY(hipMemcpy(c->u, soa.data(), soa.size() * sizeof(double), hipMemcpyHostToDevice));
	c->wStage = -1;
	return GCMX_OK;
}

gcmx_status gsx_download(gsx_ctx* c, double* aos) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!aos) return fail(GCMX_ERR_INVALID_ARG, "null layer");
	const size_t N = (size_t)c->N;
	std::vector<double> soa(kM * N);
	SX_TRY(hipStreamSynchronize(c->stream));
	if ((s = report_wait_error(c)) != GCMX_OK) return s;  // a timed-out stage made this layer
	SX_TRY(hipMemcpy(soa.data(), c->u, soa.size() * sizeof(double), hipMemcpyDeviceToHost));
	for (size_t n = 0; n < N; n++)
		for (int k = 0; k < kM; k++) aos[kM * n + k] = soa[k * N + n];
	return GCMX_OK;
}

gcmx_status gsx_set_border_plan(gsx_ctx* c, int n_cond, const int* type, const double* min_det,
                                int n, const int* nodes, const int* cond, const double* B,
                                const double* S, const signed char* outer) {
	gcmx_status s = check(c);
	if (s) return s;
	c->planGen++;  // captured step graphs point into what this call replaces
	if (n_cond < 0 || n_cond > GSX_MAX_BORDER_CONDITIONS || n < 0 || (n_cond && (!type || !min_det)) ||
	    (n && (!nodes || !cond || !B || !S || !outer)))
		return fail(GCMX_ERR_INVALID_ARG, "bad border plan");
	for (int i = 0; i < n_cond; i++)
		if (type[i] != GSX_FIXED_FORCE && type[i] != GSX_FIXED_VELOCITY)
			return fail(GCMX_ERR_INVALID_ARG, "unknown border condition type");
	for (int i = 0; i < n; i++) {
		if (nodes[i] < 0 || nodes[i] >= c->N) return fail(GCMX_ERR_INVALID_ARG, "node out of range");
		if (cond[i] < 0 || cond[i] >= n_cond) return fail(GCMX_ERR_INVALID_ARG, "condition out of range");
	}
	for (int i = 0; i < 3 * n; i++)
		if (outer[i] < 0 || outer[i] > 3) return fail(GCMX_ERR_INVALID_ARG, "bad outer code");
	SX_TRY(hipStreamSynchronize(c->stream));
	BorderDev& bd = c->bd;
	if (bd.md) SX_TRY(hipFree(bd.md));  // sized by the plan: prep_border reallocates it
	bd.md = nullptr;
	if ((s = upload(&bd.nodes, nodes, (size_t)n)) || (s = upload(&bd.cond, cond, (size_t)n)) ||
	    (s = upload(&bd.B, B, 27 * (size_t)n)) || (s = upload(&bd.S, S, 9 * (size_t)n)) ||
	    (s = upload(&bd.outer, outer, 3 * (size_t)n)))
		return s;
	std::vector<int> corrOf((size_t)c->N, -1);
	for (int i = 0; i < n; i++) {
		if (corrOf[(size_t)nodes[i]] >= 0) return fail(GCMX_ERR_INVALID_ARG, "node corrected twice");
		corrOf[(size_t)nodes[i]] = i;
	}
	std::vector<int2> nodeRec((size_t)c->N, make_int2(-1, 0));
	for (int i = 0; i < n; i++) nodeRec[(size_t)nodes[i]] = make_int2(i, cond[i]);
	if ((s = upload(&c->corrOf, corrOf.data(), corrOf.size())) ||
	    (s = upload(&bd.nodeRec, nodeRec.data(), nodeRec.size())))
		return s;
	bd.n = n;
	bd.nCond = n_cond;
	bd.args = BorderArgs{};
	bd.args.b = c->bvals;
	for (int i = 0; i < n_cond; i++) {
		bd.args.type[i] = type[i];
		for (int st = 0; st < 3; st++) bd.args.minDet[i][st] = min_det[i * 3 + st];
	}
	if ((s = upload(&bd.argsDev, &bd.args, 1))) return s;
	bd.set = true;
	bd.valuesSet = (n_cond == 0);
	return prep_border(c);
}

gcmx_status gsx_set_border_values(gsx_ctx* c, const double* b) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!c->bd.set) return fail(GCMX_ERR_STATE, "border plan not set");
	if (c->bd.nCond && !b) return fail(GCMX_ERR_INVALID_ARG, "null border values");
	// written by a one-block kernel whose arguments carry the values: ordered on
	// the context stream before the step that reads them, with no host buffer
	// that must outlive the call
	// (skipped when the values equal the ones already written: constant conditions)
	if (c->bd.nCond) {
		BorderValues v{};
		for (int i = 0; i < 3 * c->bd.nCond; i++) v.b[i] = b[i];
		if (!c->bd.valuesSet || std::memcmp(v.b, c->bd.lastValues, sizeof(v.b)) != 0) {
			SX_LAUNCH(c, k_sx_set_border_values, dim3(1), dim3(64), 0, c->stream, c->bvals, v,
			                   3 * c->bd.nCond);
			SX_TRY(hipGetLastError());
			std::memcpy(c->bd.lastValues, v.b, sizeof(v.b));
		}
	}
	c->bd.valuesSet = true;
	return GCMX_OK;
}

gcmx_status gsx_plain_correction(gsx_ctx* c) {
	gcmx_status s = check(c);
	if (s) return s;
	const BorderDev& bd = c->bd;
	if (!bd.set || !bd.valuesSet) return fail(GCMX_ERR_STATE, "border plan / values not set");
	if (c->matsSet) {  // fused with the first stage's beforeStage (the next call is stage 0)
		SX_LAUNCH(c, k_sx_begin, dim3((c->N + 255) / 256), dim3(256), 0, c->stream, c->u, c->w,
		                   c->mats, bd.n ? bd.nodeRec : nullptr, bd.S, c->N, bd.argsDev);
		c->wStage = 0;
	} else if (bd.n) {
		SX_LAUNCH(c, k_sx_plain, dim3((bd.n + 63) / 64), dim3(64), 0, c->stream, bd.nodes,
		                   bd.cond, bd.S, c->u, bd.n, c->N, bd.argsDev);
		c->wStage = -1;
	}
	SX_TRY(hipGetLastError());
	return GCMX_OK;
}

namespace {
// Node-kernel layout (gsx_set_node_lanes): eight lanes per node below kL8MaxNodes vertices.
// Measured: 32^3 meshes (35 937 vertices) run 7-35 % faster with eight lanes,
// 64^3 (274 625) 6-12 % slower.
int node_lanes(const gsx_ctx* c) { return c->nodeLanes ? c->nodeLanes : (c->N < kL8MaxNodes ? kL : 1); }
// The next stage's U for the fused beforeStage, or null after the last stage of
// the step (the next step starts with the plain corrections, which change u).
const double* nextU(const gsx_ctx* c, int stage) {
	return stage < 2 ? c->mats + (stage + 1) * 81 : nullptr;
}
}  // namespace

}  // extern "C"

namespace {
// gsx_stage_nodes' launches; with `fuse` (gsx_stage: nothing runs between the
// border and inner halves) an eligible stage runs both halves as one launch
// (k_sx_stage_l8) and *fused says so, so the finish skips the inner launch.
gcmx_status stage_nodes(gsx_ctx* c, int stage, bool fuse, bool* fused) {
	*fused = false;
	gcmx_status s = check(c);
	if (s) return s;
	if (stage < 0 || stage > 2) return fail(GCMX_ERR_INVALID_ARG, "stage out of range");
	if (!c->matsSet || !c->gradSet || !c->st[stage].set)
		return fail(GCMX_ERR_STATE, "simplex matrices / gradient plan / stage plan not set");
	const BorderDev& bd = c->bd;
	if (bd.set && bd.n && !bd.valuesSet) return fail(GCMX_ERR_STATE, "border values not set");
	const int N = c->N;
	const dim3 blk(256), grd((N + 255) / 256);
	const StageDev& st = c->st[stage];
	const bool l8 = node_lanes(c) == kL;
	// beforeStage: the invariants come from the previous stage's final writers when
	// chained, otherwise from a transform pass
	if (c->wStage != stage)
		SX_LAUNCH(c, k_sx_transform<true>, grd, blk, 0, c->stream, c->u, c->w,
		                   c->mats + stage * 81, N);
	c->wStage = -1;
	// one-launch stage (k_sx_stage_l8: gradient, border and inner groups side by side)
	// for grids of at most kFuseMaxBlocks (4096) blocks, where it measured faster
	// (32^3 meshes: 1 120 blocks); at 64^3 with eight lanes, 8 600 blocks of waiting
	// groups measured 1.45x slower than separate launches.  Mode 3 (tuning only)
	// lifts the cap.
	const size_t nblk =
	    ((size_t)((c->fuseMode == 2 ? N : 0) + st.nBorder + st.nInner) * kL + kL8Block - 1) / kL8Block;
	bool one = fuse && l8 && c->fuseMode && st.fusable && st.nBorder > 0 && st.nInner > 0 &&
	           (nblk <= kFuseMaxBlocks || c->fuseMode == 3);
	const bool withGrad = c->fuseMode == 2;  // the gradient groups in the same launch
	if (one) {  // a graph being captured would replay a stale epoch
		hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
		SX_TRY(hipStreamIsCapturing(c->stream, &cs));
		one = cs == hipStreamCaptureStatusNone;
	}
	if (one) {
		if (c->epoch == INT_MAX) {  // flags restart from zero
			SX_TRY(hipMemsetAsync(c->ready, 0, (size_t)N * sizeof(int), c->stream));
			c->epoch = 0;
		}
		const BorderDevArgs bp = {c->corrOf, (bd.set && bd.n) ? bd.cond : nullptr, bd.B, bd.S,
		                          bd.outer, bd.n, bd.nCond, st.rec, st.recB, st.recMd};
		const int ngBlk = withGrad ? (int)(((size_t)N * kL + kL8Block - 1) / kL8Block) : 0;
		// the counter wraps like the target; both advance only with a launched grid
		const unsigned target = c->gTarget + (unsigned)ngBlk;
		const StageWait sw{c->ready,      withGrad ? reinterpret_cast<unsigned*>(c->ready + N) : nullptr,
		                   target,        c->epoch + 1,
		                   c->ready + N + 1, c->waitBudget,
		                   reinterpret_cast<unsigned*>(c->ready + N + 2), c->tickets};
		if (!withGrad)
			SX_LAUNCH(c, k_sx_gradient_l8, dim3(((size_t)N * kL + kL8Block - 1) / kL8Block), dim3(kL8Block), 0,
			                   c->stream, c->w, c->grad, c->gOff, c->gNb, c->coords, c->gW, c->gM, c->gDet, N);
		const int nbBlk = (int)(((size_t)st.nBorder * kL + kL8Block - 1) / kL8Block);
		const int niBlk = (int)(((size_t)st.nInner * kL + kL8Block - 1) / kL8Block);
		SX_LAUNCH(c, k_sx_stage_l8, dim3(ngBlk + nbBlk + niBlk), dim3(kL8Block), 0, c->stream, st.border,
		                   st.nBorder, st.inner, st.nInner, nbBlk, st.fv, st.flam, st.fmeta, st.shift, c->coords,
		                   c->w, c->grad, c->wn, c->deferred, bp, bd.argsDev, c->mats + stage * 81,
		                   c->mats + 3 * 81 + stage * 81, nextU(c, stage), c->un, c->wnext, stage, N, sw, ngBlk,
		                   c->grad, c->gOff, c->gNb, c->gW, c->gM, c->gDet);
		SX_TRY(hipGetLastError());
		c->gTarget = target;
		c->tickets += (unsigned)(ngBlk + nbBlk + niBlk);
		c->epoch++;
		*fused = true;
		return GCMX_OK;
	}
	if (l8)
		SX_LAUNCH(c, k_sx_gradient_l8, dim3(((size_t)N * kL + kL8Block - 1) / kL8Block), dim3(kL8Block), 0,
		                   c->stream, c->w,
		                   c->grad, c->gOff, c->gNb, c->coords, c->gW, c->gM, c->gDet, N);
	else
		SX_LAUNCH(c, k_sx_gradient, grd, blk, 0, c->stream, c->w, c->grad, c->gOff, c->gNb,
		                   c->coords, c->gW, c->gM, c->gDet, N);
	if (st.nBorder) {
		const BorderDevArgs bp = {c->corrOf, (bd.set && bd.n) ? bd.cond : nullptr, bd.B, bd.S,
		                          bd.outer, bd.n, bd.nCond, st.rec, st.recB, st.recMd};
		if (l8) {
#ifdef GCMX_SX_DIAG_TWICE  // tuning builds only: a second, warm-cache launch of the same kernel
			for (int rep = 0; rep < 2; rep++)
#endif
#ifdef GCMX_SX_DIAG_ASINNER  // tuning builds only: time the inner kernel over the border list
			if (true)
				SX_LAUNCH(c, k_sx_inner_l8, dim3(((size_t)st.nBorder * kL + kL8Block - 1) / kL8Block),
			                   dim3(kL8Block), 0, c->stream, st.border, st.nBorder, st.fv, st.flam, st.fmeta,
			                   st.shift, c->coords, c->w, c->grad, c->wn, c->mats + 3 * 81 + stage * 81,
			                   nextU(c, stage), c->un, c->wnext, N, 0, st.nBorder + st.nInner);
			else
#endif
			SX_LAUNCH(c, k_sx_border_l8, dim3(((size_t)st.nBorder * kL + kL8Block - 1) / kL8Block),
			                   dim3(kL8Block), 0, c->stream,
			                   st.border, st.nBorder, st.fv, st.flam, st.fmeta, st.shift, c->coords, c->w,
			                   c->grad, c->wn, c->deferred, bp, bd.argsDev, c->mats + stage * 81,
			                   c->mats + 3 * 81 + stage * 81, nextU(c, stage), c->un, c->wnext, stage, N, 0,
			                   st.nBorder + st.nInner);
		}
		else  // border lists are short (a surface): 64-thread blocks spread them over the CUs
			SX_LAUNCH(c, k_sx_border, dim3((st.nBorder + 63) / 64), dim3(64), 0, c->stream, st.border,
			                   st.nBorder, st.fv, st.flam, st.fmeta, st.shift, c->coords, c->w, c->grad,
			                   c->wn, c->deferred, bp, bd.argsDev, c->mats + stage * 81,
			                   c->mats + 3 * 81 + stage * 81, nextU(c, stage), c->un, c->wnext, stage, N, 0,
			                   st.nBorder + st.nInner);
	}
	SX_TRY(hipGetLastError());
	return GCMX_OK;
}

gcmx_status stage_finish(gsx_ctx* c, int stage, bool inner_done) {
	gcmx_status s = check(c);
	if (s) return s;
	if (stage < 0 || stage > 2) return fail(GCMX_ERR_INVALID_ARG, "stage out of range");
	if (!c->matsSet || !c->gradSet || !c->st[stage].set)
		return fail(GCMX_ERR_STATE, "simplex matrices / gradient plan / stage plan not set");
	const int N = c->N;
	const dim3 blk(256);
	const StageDev& st = c->st[stage];
	if (inner_done) {
	} else if (st.nInner && node_lanes(c) == kL)
		SX_LAUNCH(c, k_sx_inner_l8, dim3(((size_t)st.nInner * kL + kL8Block - 1) / kL8Block),
		                   dim3(kL8Block), 0, c->stream,
		                   st.inner, st.nInner, st.fv, st.flam, st.fmeta, st.shift, c->coords, c->w, c->grad,
		                   c->wn, c->mats + 3 * 81 + stage * 81, nextU(c, stage), c->un, c->wnext, N,
		                   st.nBorder, st.nBorder + st.nInner);
	else if (st.nInner)
		SX_LAUNCH(c, k_sx_inner, dim3((st.nInner + 255) / 256), blk, 0, c->stream, st.inner,
		                   st.nInner, st.fv, st.flam, st.fmeta, st.shift, c->coords, c->w, c->grad,
		                   c->wn, c->mats + 3 * 81 + stage * 81, nextU(c, stage), c->un, c->wnext, N,
		                   st.nBorder, st.nBorder + st.nInner);
	SX_TRY(hipGetLastError());
	std::swap(c->u, c->un);
	if (stage < 2) {
		std::swap(c->w, c->wnext);
		c->wStage = stage + 1;
	}
	return GCMX_OK;
}

}  // namespace

extern "C" {

gcmx_status gsx_stage_nodes(gsx_ctx* c, int stage) {
	bool fused;
	return stage_nodes(c, stage, false, &fused);
}

gcmx_status gsx_stage_finish(gsx_ctx* c, int stage) { return stage_finish(c, stage, false); }

gcmx_status gsx_set_stage_fusion(gsx_ctx* c, int on) {
	gcmx_status s = check(c);
	if (s) return s;
	if (on < 0 || on > 3) return fail(GCMX_ERR_INVALID_ARG, "stage fusion must be 0..3");
	c->fuseMode = on;
	return GCMX_OK;
}

gcmx_status gsx_launch_count(const gsx_ctx* c, long long* launches) {
	if (!c || !launches) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	*launches = c->launches;
	return GCMX_OK;
}

gcmx_status gsx_stage_plan_info(const gsx_ctx* c, int stage, int* fusable, int* wait_feet) {
	if (!c || !fusable || !wait_feet) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	if (stage < 0 || stage > 2 || !c->st[stage].set) return fail(GCMX_ERR_STATE, "stage plan not set");
	*fusable = c->st[stage].fusable ? 1 : 0;
	*wait_feet = c->st[stage].waitFeet;
	return GCMX_OK;
}

gcmx_status gsx_last_stage_fused(const gsx_ctx* c, int* fused) {
	if (!c || !fused) return fail(GCMX_ERR_INVALID_ARG, "null argument");
	*fused = c->lastFused ? 1 : 0;
	return GCMX_OK;
}

gcmx_status gsx_set_node_lanes(gsx_ctx* c, int lanes) {
	gcmx_status s = check(c);
	if (s) return s;
	c->planGen++;  // captured step graphs point into what this call replaces
	if (lanes != 0 && lanes != 1 && lanes != kL) return fail(GCMX_ERR_INVALID_ARG, "node lanes must be 0, 1 or 8");
	c->nodeLanes = lanes;
	return GCMX_OK;
}

gcmx_status gsx_stage(gsx_ctx* c, int stage) {
	bool fused = false;
	gcmx_status s = stage_nodes(c, stage, true, &fused);
	if (s) return s;
	c->lastFused = fused;
	return stage_finish(c, stage, fused);
}

gcmx_status gsx_contact_create(gsx_ctx* a, gsx_ctx* b, int n, const int* nodes_a,
                               const int* nodes_b, const double* normal, const double* S,
                               const signed char* code_a, const signed char* code_b,
                               const double* min_det, gsx_contact** out) {
	if (!out) return fail(GCMX_ERR_INVALID_ARG, "null output");
	*out = nullptr;
	gcmx_status s = check(a);
	if (s) return s;
	if ((s = check(b))) return s;
	if (a == b || a->device != b->device)
		return fail(GCMX_ERR_INVALID_ARG, "a contact couples two bodies on one device");
	if (n < 0 || !min_det || (n && (!nodes_a || !nodes_b || !normal || !S || !code_a || !code_b)))
		return fail(GCMX_ERR_INVALID_ARG, "bad contact plan");
	for (int i = 0; i < n; i++)
		if (nodes_a[i] < 0 || nodes_a[i] >= a->N || nodes_b[i] < 0 || nodes_b[i] >= b->N)
			return fail(GCMX_ERR_INVALID_ARG, "contact node out of range");
	for (int i = 0; i < 3 * n; i++)
		if (code_a[i] < 0 || code_a[i] > 7 || code_b[i] < 0 || code_b[i] > 7)
			return fail(GCMX_ERR_INVALID_ARG, "bad contact wave code");
	gsx_contact* c = new gsx_contact();
	c->a = a;
	c->b = b;
	c->n = n;
	for (int st = 0; st < 3; st++)
		for (int k = 0; k < 2; k++) c->minDet[st][k] = min_det[st * 2 + k];
	if ((s = upload(&c->na, nodes_a, (size_t)n)) || (s = upload(&c->nb, nodes_b, (size_t)n)) ||
	    (s = upload(&c->normal, normal, 3 * (size_t)n)) || (s = upload(&c->S, S, 9 * (size_t)n)) ||
	    (s = upload(&c->codeA, code_a, 3 * (size_t)n)) || (s = upload(&c->codeB, code_b, 3 * (size_t)n))) {
		gsx_contact_destroy(c);
		return s;
	}
	if (hipStreamSynchronize(a->stream) != hipSuccess || hipStreamSynchronize(b->stream) != hipSuccess) {
		gsx_contact_destroy(c);
		return fail(GCMX_ERR_HIP, "hipStreamSynchronize failed");
	}
	for (int i = 0; i < n; i++) {
		a->hostDeferred[(size_t)nodes_a[i]] = 1;
		b->hostDeferred[(size_t)nodes_b[i]] = 1;
	}
	a->planGen++;  // the deferred flags are reallocated below
	b->planGen++;
	if ((s = upload(&a->deferred, a->hostDeferred.data(), a->hostDeferred.size())) ||
	    (s = upload(&b->deferred, b->hostDeferred.data(), b->hostDeferred.size()))) {
		gsx_contact_destroy(c);
		return s;
	}
	if (hipEventCreateWithFlags(&c->evA, hipEventDisableTiming) != hipSuccess ||
	    hipEventCreateWithFlags(&c->evB, hipEventDisableTiming) != hipSuccess) {
		gsx_contact_destroy(c);
		return fail(GCMX_ERR_HIP, "hipEventCreate failed");
	}
	*out = c;
	return GCMX_OK;
}

void gsx_contact_destroy(gsx_contact* c) {
	if (!c) return;
	(void)hipSetDevice(c->a->device);
	void* ptrs[] = {c->na, c->nb, c->normal, c->S, c->codeA, c->codeB};
	for (void* p : ptrs)
		if (p) (void)hipFree(p);
	if (c->evA) (void)hipEventDestroy(c->evA);
	if (c->evB) (void)hipEventDestroy(c->evB);
	delete c;
}


gcmx_status gsx_contact_plain(gsx_contact* c) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null contact");
	gcmx_status s = check(c->a);
	if (s) return s;
	if (!c->n) return GCMX_OK;
	c->a->wStage = c->b->wStage = -1;  // u changes under any prepared invariants
	return onBothStreams(c, [&] {
		SX_LAUNCH(c->a, k_sx_contact_plain, dim3((c->n + 255) / 256), dim3(256), 0, c->a->stream,
		                   c->na, c->nb, c->S, c->a->u, c->b->u, c->a->N, c->b->N, c->n);
	});
}

gcmx_status gsx_contact_correct(gsx_contact* c, int stage) {
	if (!c) return fail(GCMX_ERR_INVALID_ARG, "null contact");
	gcmx_status s = check(c->a);
	if (s) return s;
	if (stage < 0 || stage > 2) return fail(GCMX_ERR_INVALID_ARG, "stage out of range");
	if (!c->a->matsSet || !c->b->matsSet) return fail(GCMX_ERR_STATE, "simplex matrices not set");
	if (!c->n) return GCMX_OK;
	const double* mA = c->a->mats;
	const double* mB = c->b->mats;
	return onBothStreams(c, [&] {
		SX_LAUNCH(c->a, k_sx_contact, dim3((c->n + 63) / 64), dim3(64), 0, c->a->stream, c->na,
		                   c->nb, c->normal, c->S, c->codeA, c->codeB, mA + stage * 81,
		                   mA + 3 * 81 + stage * 81, mB + stage * 81, mB + 3 * 81 + stage * 81,
		                   c->a->wn, c->b->wn, c->a->N, c->b->N, c->n, stage, c->minDet[stage][0],
		                   c->minDet[stage][1], nextU(c->a, stage), nextU(c->b, stage), c->a->un,
		                   c->b->un, c->a->wnext, c->b->wnext);
	});
}

namespace {
// The step body: Engine::nextTimeStep after setBorderValues (simplex/Engine.cpp:95-116,
// 119-143): plain corrections (contacts, then bodies), then per stage the bodies'
// beforeStage + contactAndBorderStage, the contact correctors, the bodies' finish.
gcmx_status step_body(const std::vector<gsx_ctx*>& bodies, const std::vector<gsx_contact*>& contacts) {
	gcmx_status s;
	for (gsx_contact* k : contacts)
		if ((s = gsx_contact_plain(k))) return s;
	for (gsx_ctx* b : bodies)
		if (b->bd.set && b->bd.n && (s = gsx_plain_correction(b))) return s;
	for (int stage = 0; stage < 3; stage++) {
		for (gsx_ctx* b : bodies)
			if ((s = gsx_stage_nodes(b, stage))) return s;
		for (gsx_contact* k : contacts)
			if ((s = gsx_contact_correct(k, stage))) return s;
		for (gsx_ctx* b : bodies)
			if ((s = gsx_stage_finish(b, stage))) return s;
	}
	return GCMX_OK;
}
}  // namespace

gcmx_status gsx_step(gsx_ctx* const* bodies_, int n_bodies, gsx_contact* const* contacts_,
                     int n_contacts) {
	if (!bodies_ || n_bodies < 1 || n_contacts < 0 || (n_contacts > 0 && !contacts_))
		return fail(GCMX_ERR_INVALID_ARG, "bad gsx_step arguments");
	std::vector<gsx_ctx*> bodies(bodies_, bodies_ + n_bodies);
	std::vector<gsx_contact*> contacts(contacts_, contacts_ + n_contacts);
	gsx_ctx* lead = bodies[0];
	gcmx_status s;
	for (gsx_ctx* b : bodies) {
		if ((s = check(b))) return s;
		if (b->device != lead->device) return fail(GCMX_ERR_INVALID_ARG, "bodies on different devices");
		if (b->bd.set && b->bd.n && !b->bd.valuesSet) return fail(GCMX_ERR_STATE, "border values not set");
	}
	for (gsx_contact* k : contacts) {
		bool in = false;
		for (gsx_ctx* b : bodies) in = in || (k && (k->a == b || k->b == b));
		if (!k || !in) return fail(GCMX_ERR_INVALID_ARG, "contact of a body outside the group");
	}
	SX_TRY(hipSetDevice(lead->device));
	std::vector<unsigned> gens;
	for (gsx_ctx* b : bodies) gens.push_back(b->planGen);
	if (!lead->graphs || lead->graphs->bodies != bodies || lead->graphs->contacts != contacts ||
	    lead->graphs->gens != gens) {
		lead->graphs.reset(new StepGraphs());
		StepGraphs& g = *lead->graphs;
		g.bodies = bodies;
		g.contacts = contacts;
		g.gens = gens;
		g.evBody.assign(bodies.size(), nullptr);
		SX_TRY(hipEventCreateWithFlags(&g.evFork, hipEventDisableTiming));
		SX_TRY(hipEventCreateWithFlags(&g.evJoin, hipEventDisableTiming));
		for (auto& e : g.evBody) SX_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	}
	StepGraphs& g = *lead->graphs;
	std::vector<BodyState> now;
	for (gsx_ctx* b : bodies) now.push_back(body_state(b));
	StepGraphs::Entry* hit = nullptr;
	for (auto& e : g.entries)
		if (e.before == now) hit = &e;
	if (!hit) {
		// Capture the step: the other bodies' streams join the capture through an
		// event of the lead stream and rejoin it at the end.  Kernels do not run
		// during capture; the host-side swaps do, and are restored afterwards.
		StepGraphs::Entry e;
		e.before = now;
		SX_TRY(hipStreamBeginCapture(lead->stream, hipStreamCaptureModeRelaxed));
		s = GCMX_OK;
		if (hipEventRecord(g.evFork, lead->stream) != hipSuccess) s = fail(GCMX_ERR_HIP, "capture fork");
		for (size_t i = 1; i < bodies.size() && !s; i++)
			if (hipStreamWaitEvent(bodies[i]->stream, g.evFork, 0) != hipSuccess) s = fail(GCMX_ERR_HIP, "capture fork");
		if (!s) s = step_body(bodies, contacts);
		for (size_t i = 1; i < bodies.size() && !s; i++)
			if (hipEventRecord(g.evBody[i], bodies[i]->stream) != hipSuccess ||
			    hipStreamWaitEvent(lead->stream, g.evBody[i], 0) != hipSuccess)
				s = fail(GCMX_ERR_HIP, "capture join");
		hipGraph_t graph = nullptr;
		const hipError_t ec = hipStreamEndCapture(lead->stream, &graph);
		for (gsx_ctx* b : bodies) e.after.push_back(body_state(b));
		for (size_t i = 0; i < bodies.size(); i++) set_body_state(bodies[i], e.before[i]);
		if (s || ec != hipSuccess || !graph) {
			if (graph) (void)hipGraphDestroy(graph);
			return s ? s : fail(GCMX_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
		}
		e.graph = graph;
		if (hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0) != hipSuccess) {
			(void)hipGraphDestroy(graph);
			return fail(GCMX_ERR_HIP, "hipGraphInstantiate failed");
		}
		g.entries.push_back(e);
		hit = &g.entries.back();
	}
	// The other bodies' pending work (border values, uploads) precedes the graph,
	// and their later work follows it.
	for (size_t i = 1; i < bodies.size(); i++) {
		SX_TRY(hipEventRecord(g.evBody[i], bodies[i]->stream));
		SX_TRY(hipStreamWaitEvent(lead->stream, g.evBody[i], 0));
	}
	SX_TRY(hipGraphLaunch(hit->exec, lead->stream));
	SX_TRY(hipEventRecord(g.evJoin, lead->stream));
	for (size_t i = 1; i < bodies.size(); i++) SX_TRY(hipStreamWaitEvent(bodies[i]->stream, g.evJoin, 0));
	for (size_t i = 0; i < bodies.size(); i++) set_body_state(bodies[i], hit->after[i]);
	return GCMX_OK;
}

gcmx_status gsx_sync(gsx_ctx* c) {
	gcmx_status s = check(c);
	if (s) return s;
	SX_TRY(hipStreamSynchronize(c->stream));
	return report_wait_error(c);
}

gcmx_status gsx_set_wait_budget(gsx_ctx* c, int polls) {
	gcmx_status s = check(c);
	if (s) return s;
	c->waitBudget = polls;
	return GCMX_OK;
}

}  // extern "C"

// ---- tests only: the device interpolation functions on given inputs -----------
namespace {
// Per case i: out[2i] = tet_hybrid (a CELL foot), out[2i + 1] = tet_linear (a
// SPACETIME foot / interpolateInOwner's value), with the gradient terms formed
// exactly as grad_dot forms them from q - c_j.
__global__ __launch_bounds__(64) void k_sx_test_interp(int n, const double* __restrict__ v,
                                                      const double* __restrict__ g, const double* __restrict__ c,
                                                      const double* __restrict__ q, const double* __restrict__ lam,
                                                      double* __restrict__ out) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	double vv[4], dots[4], l[4];
#pragma unroll
	for (int j = 0; j < 4; j++) {
		vv[j] = v[4 * i + j];
		l[j] = lam[4 * i + j];
		double d[3];
#pragma unroll
		for (int r = 0; r < 3; r++) d[r] = q[3 * i + r] - c[(4 * i + j) * 3 + r];
		const double* gj = g + (4 * i + j) * 3;
		double dot = gj[0] * d[0];
		dot += gj[1] * d[1];
		dot += gj[2] * d[2];
		dots[j] = dot;
	}
	out[2 * i] = tet_hybrid(vv, dots, l);
	out[2 * i + 1] = tet_linear(vv, l);
}
}  // namespace

extern "C" gcmx_status gsx_test_interpolate(int device, int n, const double* v, const double* g, const double* c,
                                            const double* q, const double* lam, double* out) {
	if (n < 1 || n > (1 << 20) || !v || !g || !c || !q || !lam || !out)
		return fail(GCMX_ERR_INVALID_ARG, "gsx_test_interpolate: bad arguments");
	SX_TRY(hipSetDevice(device));
	const size_t sz[6] = {4 * (size_t)n, 12 * (size_t)n, 12 * (size_t)n, 3 * (size_t)n, 4 * (size_t)n, 2 * (size_t)n};
	const double* src[5] = {v, g, c, q, lam};
	double* d[6] = {};
	gcmx_status st = GCMX_OK;
	for (int k = 0; k < 6 && st == GCMX_OK; k++) {
		if (hipMalloc(&d[k], sz[k] * sizeof(double)) != hipSuccess) st = fail(GCMX_ERR_OOM, "gsx_test_interpolate");
		else if (k < 5 && hipMemcpy(d[k], src[k], sz[k] * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
			st = fail(GCMX_ERR_HIP, "gsx_test_interpolate: upload");
	}
	if (st == GCMX_OK) {
		hipLaunchKernelGGL(k_sx_test_interp, dim3((n + 63) / 64), dim3(64), 0, 0, n, d[0], d[1], d[2], d[3], d[4], d[5]);
		if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
		    hipMemcpy(out, d[5], sz[5] * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
			st = fail(GCMX_ERR_HIP, "gsx_test_interpolate: kernel");
	}
	for (double* p : d)
		if (p) (void)hipFree(p);
	return st;
}
