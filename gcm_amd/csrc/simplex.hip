// simplex.hip -- device half of the simplex (tetrahedral) grid-characteristic
// stage in Riemann invariants (gsx_* in include/gcmx.h).
//
// One stage s (engine/simplex/Engine.cpp:117-148, GLOBAL_BASIS + PRODUCT):
//   k_sx_transform(U_s)   beforeStage: w = U_s u for every node
//                         (GridCharacteristicMethodInRiemannInvariants.hpp:44-56)
//   k_sx_gradient         Differentiation::estimateGradient of w (Differentiation.hpp:33-63)
//   k_sx_nodes(border)    contactAndBorderStage (hpp:57-95)
//   k_sx_nodes(inner)     innerStage (hpp:98-112) -- space-time feet read the border
//                         nodes' new invariants written by the previous launch
//   k_sx_transform(U1_s)  afterStage: u_new = U1_s w_new (hpp:115-126), then swap.
// Storage is SoA: component c of node n at [c * N + n]; gradients [r][c][n].
// Arithmetic follows the reference expression by expression (-ffp-contract=off).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gcmx.h"
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

struct StageDev {
	gsx_foot* feet = nullptr;
	int* border = nullptr;
	int* inner = nullptr;
	int nBorder = 0, nInner = 0;
	bool set = false;
};

}  // namespace

struct gsx_ctx {
	int device = 0, N = 0;
	hipStream_t stream = nullptr;
	double *coords = nullptr, *u = nullptr, *un = nullptr, *w = nullptr, *wn = nullptr,
	       *grad = nullptr;
	double* mats = nullptr;  // [2][3][81]: U then U1
	bool matsSet = false;
	int *gOff = nullptr, *gNb = nullptr;
	double *gRows = nullptr, *gW = nullptr, *gM = nullptr, *gDet = nullptr;
	bool gradSet = false;
	StageDev st[3];
};

namespace {

// out[c] = M(c,0) in[0] + sum_{j>=1} M(c,j) in[j]  (linal/operators.hpp:109-123)
__global__ __launch_bounds__(256) void k_sx_transform(const double* __restrict__ in,
                                                      double* __restrict__ out,
                                                      const double* __restrict__ Mx, int N) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	double v[kM];
#pragma unroll
	for (int j = 0; j < kM; j++) v[j] = in[j * N + n];
#pragma unroll
	for (int c = 0; c < kM; c++) {
		double s = Mx[c * kM + 0] * v[0];
#pragma unroll
		for (int j = 1; j < kM; j++) s += Mx[c * kM + j] * v[j];
		out[c * N + n] = s;
	}
}

__device__ __forceinline__ double det3(double m11, double m12, double m13, double m21, double m22,
                                       double m23, double m31, double m32, double m33) {
	return m11 * (m22 * m33 - m23 * m32) - m12 * (m21 * m33 - m23 * m31) +
	       m13 * (m21 * m32 - m22 * m31);
}

// linearLeastSquares(A, b, W) = solve(A^T W A, A^T (W b)) per component, with
// transposeMultiply's order (first term, then +=) over all kMaxNb rows: the
// unused rows are zero rows and add +0.
__global__ __launch_bounds__(256) void k_sx_gradient(const double* __restrict__ w,
                                                     double* __restrict__ grad,
                                                     const int* __restrict__ off,
                                                     const int* __restrict__ nbs,
                                                     const double* __restrict__ rows,
                                                     const double* __restrict__ wts,
                                                     const double* __restrict__ Mm,
                                                     const double* __restrict__ dets, int N) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	const int b0 = off[n], K = off[n + 1] - b0;
	const double* M = Mm + 9 * n;
	const double det = dets[n];
	for (int c = 0; c < kM; c++) {
		const double wc = w[c * N + n];
		double r0 = 0, r1 = 0, r2 = 0;
		for (int i = 0; i < K; i++) {
			const int e = b0 + i;
			const double bi = w[c * N + nbs[e]] - wc;  // b(i) = pde(neighbor) - pde(it)
			const double wb = wts[e] * bi;             // (W * b)(i)
			const double t0 = rows[3 * e + 0] * wb, t1 = rows[3 * e + 1] * wb,
			             t2 = rows[3 * e + 2] * wb;
			if (i == 0) {
				r0 = t0; r1 = t1; r2 = t2;
			} else {
				r0 += t0; r1 += t1; r2 += t2;
			}
		}
		if (K < kMaxNb) {  // the zero rows: 0 * (0 * 0) = +0
			r0 += 0.0; r1 += 0.0; r2 += 0.0;
		}
		const double d1 = det3(r0, M[1], M[2], r1, M[4], M[5], r2, M[7], M[8]);
		const double d2 = det3(M[0], r0, M[2], M[3], r1, M[5], M[6], r2, M[8]);
		const double d3 = det3(M[0], M[1], r0, M[3], M[4], r1, M[6], M[7], r2);
		grad[(0 * kM + c) * N + n] = d1 / det;
		grad[(1 * kM + c) * N + n] = d2 / det;
		grad[(2 * kM + c) * N + n] = d3 / det;
	}
}

__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

// interpolateValuesAround (hpp:156-198) for the listed nodes, feet resolved on the host.
__global__ __launch_bounds__(256) void k_sx_nodes(const int* __restrict__ nodes, int count,
                                                  const gsx_foot* __restrict__ feet,
                                                  const double* __restrict__ coords,
                                                  const double* __restrict__ w,
                                                  const double* __restrict__ grad,
                                                  double* __restrict__ wn, int N) {
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= count) return;
	const int n = nodes[t];
	for (int k = 0; k < kM; k++) {
		double ans;
		if (k >= 6) {
			ans = w[k * N + n];  // dx(k) == 0: exact hit (hpp:166-170)
		} else {
			const gsx_foot& f = feet[(size_t)n * 6 + k];
			if (f.kind == GSX_FOOT_CELL) {
				// TetrahedronInterpolator::hybridInterpolate (hpp:93-104)
				double v[4], term[4];
#pragma unroll
				for (int i = 0; i < 4; i++) {
					const int p = f.v[i];
					v[i] = w[k * N + p];
					const double d0 = f.q[0] - coords[0 * N + p];
					const double d1 = f.q[1] - coords[1 * N + p];
					const double d2 = f.q[2] - coords[2 * N + p];
					double dot = grad[(0 * kM + k) * N + p] * d0;
					dot += grad[(1 * kM + k) * N + p] * d1;
					dot += grad[(2 * kM + k) * N + p] * d2;
					term[i] = v[i] + dot / 2.0;
				}
				const double quadratic =
				    f.lam[0] * term[0] + f.lam[1] * term[1] + f.lam[2] * term[2] + f.lam[3] * term[3];
				const double mn = std_min(std_min(std_min(v[0], v[1]), v[2]), v[3]);
				const double mx = std_max(std_max(std_max(v[0], v[1]), v[2]), v[3]);
				const double limited = std_min(std_max(quadratic, mn), mx);
				ans = (quadratic == limited)
				          ? quadratic
				          : f.lam[0] * v[0] + f.lam[1] * v[1] + f.lam[2] * v[2] + f.lam[3] * v[3];
			} else if (f.kind == GSX_FOOT_SPACETIME) {
				double val[4];
#pragma unroll
				for (int i = 0; i < 4; i++) {
					const int s = f.slot[i];
					val[i] = (s < 3) ? w[k * N + f.v[s]] : wn[k * N + f.v[s - 3]];
				}
				ans = f.lam[0] * val[0] + f.lam[1] * val[1] + f.lam[2] * val[2] + f.lam[3] * val[3];
			} else {
				ans = 0.0;  // outer invariant / walk ended on a vertex
			}
		}
		wn[k * N + n] = ans;
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
	std::vector<double> soa(3 * N);
	for (size_t n = 0; n < N; n++)
		for (int r = 0; r < 3; r++) soa[r * N + n] = coords[3 * n + r];
	gcmx_status s = upload(&c->coords, soa.data(), 3 * N);
	if (s) { gsx_destroy(c); return s; }
	double** bufs[5] = {&c->u, &c->un, &c->w, &c->wn, &c->grad};
	const size_t sizes[5] = {kM * N, kM * N, kM * N, kM * N, 3 * kM * N};
	for (int i = 0; i < 5; i++) {
		if (hipMalloc(bufs[i], sizes[i] * sizeof(double)) != hipSuccess ||
		    hipMemset(*bufs[i], 0, sizes[i] * sizeof(double)) != hipSuccess) {
			gsx_destroy(c);
			return fail(GCMX_ERR_OOM, "simplex layer allocation failed");
		}
	}
	*out = c;
	return GCMX_OK;
}

void gsx_destroy(gsx_ctx* c) {
	if (!c) return;
	(void)hipSetDevice(c->device);
	if (c->stream) (void)hipStreamSynchronize(c->stream);
	void* ptrs[] = {c->coords, c->u, c->un, c->w, c->wn, c->grad, c->mats, c->gOff, c->gNb,
	                c->gRows, c->gW, c->gM, c->gDet};
	for (void* p : ptrs)
		if (p) (void)hipFree(p);
	for (auto& st : c->st) {
		if (st.feet) (void)hipFree(st.feet);
		if (st.border) (void)hipFree(st.border);
		if (st.inner) (void)hipFree(st.inner);
	}
	if (c->stream) (void)hipStreamDestroy(c->stream);
	delete c;
}

gcmx_status gsx_set_matrices(gsx_ctx* c, const double* U, const double* U1) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!U || !U1) return fail(GCMX_ERR_INVALID_ARG, "null matrices");
	std::vector<double> m(2 * 3 * 81);
	std::memcpy(m.data(), U, 3 * 81 * sizeof(double));
	std::memcpy(m.data() + 3 * 81, U1, 3 * 81 * sizeof(double));
	SX_TRY(hipStreamSynchronize(c->stream));
	s = upload(&c->mats, m.data(), m.size());
	if (s) return s;
	c->matsSet = true;
	return GCMX_OK;
}

gcmx_status gsx_set_gradient_plan(gsx_ctx* c, const int* off, const int* nbs, const double* rows,
                                  const double* wts, const double* M, const double* det) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!off || !M || !det) return fail(GCMX_ERR_INVALID_ARG, "null gradient plan");
	const int N = c->N, E = off[N];
	if (off[0] != 0 || E < 0) return fail(GCMX_ERR_INVALID_ARG, "bad gradient offsets");
	for (int n = 0; n < N; n++) {
		const int K = off[n + 1] - off[n];
		if (K < 1 || K > kMaxNb) return fail(GCMX_ERR_INVALID_ARG, "1..20 neighbours per node expected");
		if (!(det[n] != 0)) return fail(GCMX_ERR_INVALID_ARG, "singular gradient system");
	}
	for (int e = 0; e < E; e++)
		if (nbs[e] < 0 || nbs[e] >= N) return fail(GCMX_ERR_INVALID_ARG, "neighbour out of range");
	SX_TRY(hipStreamSynchronize(c->stream));
	if ((s = upload(&c->gOff, off, (size_t)N + 1)) || (s = upload(&c->gNb, nbs, (size_t)E)) ||
	    (s = upload(&c->gRows, rows, 3 * (size_t)E)) || (s = upload(&c->gW, wts, (size_t)E)) ||
	    (s = upload(&c->gM, M, 9 * (size_t)N)) || (s = upload(&c->gDet, det, (size_t)N)))
		return s;
	c->gradSet = true;
	return GCMX_OK;
}

gcmx_status gsx_set_stage_plan(gsx_ctx* c, int stage, const gsx_foot* feet, int nb,
                               const int* border, int ni, const int* inner) {
	gcmx_status s = check(c);
	if (s) return s;
	if (stage < 0 || stage > 2 || !feet || nb < 0 || ni < 0 || (nb && !border) || (ni && !inner))
		return fail(GCMX_ERR_INVALID_ARG, "bad stage plan");
	const int N = c->N;
	for (int i = 0; i < nb; i++)
		if (border[i] < 0 || border[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "node out of range");
	for (int i = 0; i < ni; i++)
		if (inner[i] < 0 || inner[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "node out of range");
	for (size_t e = 0; e < (size_t)N * 6; e++) {
		const gsx_foot& f = feet[e];
		const int nv = f.kind == GSX_FOOT_CELL ? 4 : f.kind == GSX_FOOT_SPACETIME ? 3 : 0;
		if (f.kind < 0 || f.kind > 3) return fail(GCMX_ERR_INVALID_ARG, "bad foot kind");
		for (int i = 0; i < nv; i++)
			if (f.v[i] < 0 || f.v[i] >= N) return fail(GCMX_ERR_INVALID_ARG, "foot vertex out of range");
		if (f.kind == GSX_FOOT_SPACETIME)
			for (int i = 0; i < 4; i++)
				if (f.slot[i] < 0 || f.slot[i] > 5) return fail(GCMX_ERR_INVALID_ARG, "bad slot");
	}
	SX_TRY(hipStreamSynchronize(c->stream));
	StageDev& st = c->st[stage];
	if ((s = upload(&st.feet, feet, (size_t)N * 6)) || (s = upload(&st.border, border, (size_t)nb)) ||
	    (s = upload(&st.inner, inner, (size_t)ni)))
		return s;
	st.nBorder = nb;
	st.nInner = ni;
	st.set = true;
	return GCMX_OK;
}

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
	return GCMX_OK;
}

gcmx_status gsx_download(gsx_ctx* c, double* aos) {
	gcmx_status s = check(c);
	if (s) return s;
	if (!aos) return fail(GCMX_ERR_INVALID_ARG, "null layer");
	const size_t N = (size_t)c->N;
	std::vector<double> soa(kM * N);
	SX_TRY(hipStreamSynchronize(c->stream));
	SX_TRY(hipMemcpy(soa.data(), c->u, soa.size() * sizeof(double), hipMemcpyDeviceToHost));
	for (size_t n = 0; n < N; n++)
		for (int k = 0; k < kM; k++) aos[kM * n + k] = soa[k * N + n];
	return GCMX_OK;
}

gcmx_status gsx_stage(gsx_ctx* c, int stage) {
	gcmx_status s = check(c);
	if (s) return s;
	if (stage < 0 || stage > 2) return fail(GCMX_ERR_INVALID_ARG, "stage out of range");
	if (!c->matsSet || !c->gradSet || !c->st[stage].set)
		return fail(GCMX_ERR_STATE, "simplex matrices / gradient plan / stage plan not set");
	const int N = c->N;
	const dim3 blk(256), grd((N + 255) / 256);
	const StageDev& st = c->st[stage];
	hipLaunchKernelGGL(k_sx_transform, grd, blk, 0, c->stream, c->u, c->w, c->mats + stage * 81, N);
	hipLaunchKernelGGL(k_sx_gradient, grd, blk, 0, c->stream, c->w, c->grad, c->gOff, c->gNb,
	                   c->gRows, c->gW, c->gM, c->gDet, N);
	if (st.nBorder)
		hipLaunchKernelGGL(k_sx_nodes, dim3((st.nBorder + 255) / 256), blk, 0, c->stream, st.border,
		                   st.nBorder, st.feet, c->coords, c->w, c->grad, c->wn, N);
	if (st.nInner)
		hipLaunchKernelGGL(k_sx_nodes, dim3((st.nInner + 255) / 256), blk, 0, c->stream, st.inner,
		                   st.nInner, st.feet, c->coords, c->w, c->grad, c->wn, N);
	hipLaunchKernelGGL(k_sx_transform, grd, blk, 0, c->stream, c->wn, c->un,
	                   c->mats + 3 * 81 + stage * 81, N);
	SX_TRY(hipGetLastError());
	std::swap(c->u, c->un);
	return GCMX_OK;
}

gcmx_status gsx_sync(gsx_ctx* c) {
	gcmx_status s = check(c);
	if (s) return s;
	SX_TRY(hipStreamSynchronize(c->stream));
	return GCMX_OK;
}

}  // extern "C"
