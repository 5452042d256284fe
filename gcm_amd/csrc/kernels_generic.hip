// kernels_generic.hip -- the any-configuration stage kernel and layout kernels.
//
// k_stage_generic: one thread per inner node, any dimensionality, borderSize
// and per-node material.  It is GridCharacteristicMethod<Mesh>::stage
// (engine/cubic/GridCharacteristicMethod.hpp:42-52) with two exact
// simplifications: a product with an exact-zero matrix entry is skipped (the
// reference adds it; x + 0*y == x for finite y), and only the components a
// non-zero U entry asks for are interpolated (the per-component interpolation
// is independent).  Summation order of the remaining terms is the reference's
// (linal/functions.hpp:254-267, linal/operators.hpp:109-123).
#include "common.hpp"
#include "launch.hpp"

namespace gcmx {

template <int D, int BS, bool HETERO>
__global__ __launch_bounds__(256) void k_stage_generic(const double* __restrict__ cur,
                                                       double* __restrict__ nxt, Geo g, int s,
                                                       const AxisTable* __restrict__ tabs,
                                                       const uint8_t* __restrict__ mat) {
	constexpr int M = pde_size(D);
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= g.n_inner) return;
	const int z = (int)(i % g.sizes[2]);
	const long long t = i / g.sizes[2];
	const int y = (int)(t % g.sizes[1]);
	const int x = (int)(t / g.sizes[1]);
	const long long off = g.origin + x * g.stride[0] + y * g.stride[1] + z * g.stride[2];
	const AxisTable& T = tabs[(HETERO ? (int)mat[i] : 0) * D + s];
	const long long st = g.stride[s];

	double r[M];
#pragma unroll
	for (int k = 0; k < M; k++) {
		const long long step = T.shift[k] * st;
		const int kf = T.kf[k];
		const bool zq = T.zero_q[k] != 0;
		double acc = 0.0;
		bool first = true;
#pragma unroll
		for (int j = 0; j < M; j++) {
			const double u = T.U[k * M + j];
			if (u != 0.0) {
				const double* p = cur + j * g.cs + off;
				double v;
				if (zq) {
					v = p[0];
				} else {
					double sv[BS + 1];
#pragma unroll
					for (int a = 0; a <= BS; a++) sv[a] = p[a * step];
					v = newton_minmax<BS>(sv, kf, T.coef[k]);
				}
				acc = first ? u * v : acc + u * v;
				first = false;
			}
		}
		r[k] = acc;
	}
#pragma unroll
	for (int c = 0; c < M; c++) {
		double acc = 0.0;
		bool first = true;
#pragma unroll
		for (int n = 0; n < M; n++) {
			const double w = T.U1[c * M + n];
			if (w != 0.0) {
				acc = first ? w * r[n] : acc + w * r[n];
				first = false;
			}
		}
		nxt[c * g.cs + off] = acc;
	}
}

// Parity-random field: SplitMix64 over global (x,y,z,c).
__device__ __forceinline__ double splitmix_uniform(uint64_t seed, uint64_t n) {
	uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	z = z ^ (z >> 31);
	return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

__global__ __launch_bounds__(256) void k_fill_random(double* __restrict__ cur, Geo g,
                                                     int gx0, int gy0, int gz0,
                                                     long long GY, long long GZ,
                                                     uint64_t seed) {
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= g.n_inner) return;
	const int z = (int)(i % g.sizes[2]);
	const long long t = i / g.sizes[2];
	const int y = (int)(t % g.sizes[1]);
	const int x = (int)(t / g.sizes[1]);
	const long long off = g.origin + x * g.stride[0] + y * g.stride[1] + z * g.stride[2];
	const uint64_t base =
	    (((uint64_t)(x + gx0) * (uint64_t)GY + (uint64_t)(y + gy0)) * (uint64_t)GZ +
	     (uint64_t)(z + gz0)) * (uint64_t)g.M;
	for (int c = 0; c < g.M; c++) cur[c * g.cs + off] = splitmix_uniform(seed, base + c);
}

// Copy a box of nodes between two layers (ContactCopier::apply,
// engine/cubic/ContactConditions.hpp:56-68).  Box given in local multi-indices.
__global__ __launch_bounds__(256) void k_copy_box(double* __restrict__ dst, Geo gd,
                                                  const double* __restrict__ src, Geo gs,
                                                  int dx0, int dy0, int dz0, int sx0, int sy0,
                                                  int sz0, int ex, int ey, int ez) {
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	const long long n = (long long)ex * ey * ez;
	if (i >= n) return;
	const int z = (int)(i % ez);
	const long long t = i / ez;
	const int y = (int)(t % ey);
	const int x = (int)(t / ey);
	const long long od = gd.origin + (x + dx0) * gd.stride[0] + (y + dy0) * gd.stride[1] +
	                     (z + dz0) * gd.stride[2];
	const long long os = gs.origin + (x + sx0) * gs.stride[0] + (y + sy0) * gs.stride[1] +
	                     (z + sz0) * gs.stride[2];
	for (int c = 0; c < gd.M; c++) dst[c * gd.cs + od] = src[c * gs.cs + os];
}

// cubic::BorderConditions::handleBorderPoint (engine/cubic/BorderConditions.hpp:94-114)
// for a list of face nodes.  quantity codes: PhysicalQuantities::T.
__host__ __device__ __forceinline__ int quantity_component(int D, int q) {
	// Vx..Vz = 2..4 ; Sxx,Sxy,Sxz,Syy,Syz,Szz = 5..10 (VelocitySigmaVariables.cpp:51-66)
	if (q >= 2 && q <= 4) return (q - 2) < D ? q - 2 : -1;
	if (q >= 5 && q <= 10) {
		const int ii[6] = {0, 0, 0, 1, 1, 2};
		const int jj[6] = {0, 1, 2, 1, 2, 2};
		const int i = ii[q - 5], j = jj[q - 5];
		if (i >= D || j >= D) return -1;
		return D + (i * D - ((i - 1) * i) / 2 + j - i);
	}
	return -1;
}

// One border node: its bs ghost nodes along `axis` become the mirrored inner
// nodes, then the condition's quantities are applied in order (std::map order in
// the reference): ghost = -inner + 2 f(t); PRESSURE clears the vector and sets
// the diagonal stresses.  base: element offset of the border node.
__device__ __forceinline__ void border_point(double* __restrict__ cur, const Geo& g, long long base,
                                             int axis, int inner_sign, const BorderQ& bq) {
	const int D = g.D, M = g.M;
	const long long st = g.stride[axis];
	for (int a = 1; a <= g.bs; a++) {
		const long long oi = base + inner_sign * a * st;
		const long long og = base - inner_sign * a * st;
		double v[kMaxM];
		for (int c = 0; c < M; c++) v[c] = cur[c * g.cs + oi];
		double w[kMaxM];
		for (int c = 0; c < M; c++) w[c] = v[c];
		for (int k = 0; k < bq.n; k++) {
			const int q = bq.q[k];
			const double two_f = 2 * bq.v[k];
			if (q == 12) {  // PRESSURE: get = -trace/D ; set clears the vector
				double tr = 0;
				for (int d = 0; d < D; d++) tr += v[D + (d * D - ((d - 1) * d) / 2)];
				const double inner_value = (-tr) / D;
				const double gv = -inner_value + two_f;
				for (int c = 0; c < M; c++) w[c] = 0.0;
				for (int d = 0; d < D; d++) w[D + (d * D - ((d - 1) * d) / 2)] = -gv;
			} else {
				const int c = quantity_component(D, q);
				if (c < 0) continue;
				w[c] = -v[c] + two_f;
			}
		}
		for (int c = 0; c < M; c++) cur[c * g.cs + og] = w[c];
	}
}

// A list of face nodes (D ints each, device-resident).  Nodes of one face are
// distinct and each thread owns its node's ghost column: no races.
__global__ __launch_bounds__(64) void k_border_fill(double* __restrict__ cur, Geo g, int axis,
                                                    int inner_sign, int n_nodes,
                                                    const int* __restrict__ nodes, BorderQ bq) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_nodes) return;
	long long base = g.origin;
	for (int d = 0; d < g.D; d++) base += (long long)nodes[i * g.D + d] * g.stride[d];
	border_point(cur, g, base, axis, inner_sign, bq);
}

// Every node of the face (axis, side): the inner extent of the other axes, the
// fastest remaining axis on the thread index (coalesced for the x and y faces).
__global__ __launch_bounds__(256) void k_face_fill(double* __restrict__ cur, Geo g, int axis,
                                                   int side, BorderQ bq) {
	int ext[2] = {1, 1}, ax[2] = {0, 0}, n = 0;
	for (int d = 0; d < g.D; d++)
		if (d != axis) {
			ax[n] = d;
			ext[n] = g.sizes[d];
			n++;
		}
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= (long long)ext[0] * ext[1]) return;
	long long base = g.origin + (long long)(side > 0 ? g.sizes[axis] - 1 : 0) * g.stride[axis];
	if (n == 1) base += i * g.stride[ax[0]];
	if (n == 2) base += (i / ext[1]) * g.stride[ax[0]] + (i % ext[1]) * g.stride[ax[1]];
	border_point(cur, g, base, axis, side > 0 ? -1 : 1, bq);
}

// The same for 3-D isotropic elasticity (9 components) and a condition without
// PRESSURE, as (mask, 2 f(t)) per component -- the last setting of a component
// wins, as in the quantity loop above: every component in registers, no
// dynamically indexed arrays (the generic form keeps them in scratch memory);
// one thread per (face node, component): blockIdx.y = the component.
__global__ __launch_bounds__(256) void k_face_fill9(double* __restrict__ cur, Geo g, int axis, int side,
                                                    FaceCond fc) {
	const int a0 = axis == 0 ? 1 : 0, a1 = axis == 2 ? 1 : 2;  // the other two axes, last fastest
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	const long long n1 = g.sizes[a1];
	if (i >= (long long)g.sizes[a0] * n1) return;
	const long long base = g.origin + (long long)(side > 0 ? g.sizes[axis] - 1 : 0) * g.stride[axis] +
	                       (i / n1) * g.stride[a0] + (i % n1) * g.stride[a1];
	const int inner_sign = side > 0 ? -1 : 1;
	const long long st = g.stride[axis];
	const int c = blockIdx.y;
	const bool set = (fc.mask >> c) & 1u;
	double two = 0.0;
#pragma unroll
	for (int k = 0; k < 9; k++)
		if (k == c) two = fc.two_v[k];
	double* p = cur + (long long)c * g.cs;
	for (int a = 1; a <= g.bs; a++) {
		const double v = p[base + inner_sign * a * st];
		p[base - inner_sign * a * st] = set ? -v + two : v;
	}
}

// Every node of the face with a per-node condition map (gcmx_face_map): node i
// (the other axes' inner indices, last fastest) takes condition bq[map[i]]; a
// node no condition covers keeps its ghosts (BorderConditions::apply visits only
// the nodes of its conditions, BorderConditions.hpp:81-91).
__global__ __launch_bounds__(256) void k_face_fill_map(double* __restrict__ cur, Geo g, int axis, int side,
                                                       const uint8_t* __restrict__ map,
                                                       const BorderQ* __restrict__ bq) {
	int ext[2] = {1, 1}, ax[2] = {0, 0}, n = 0;
	for (int d = 0; d < g.D; d++)
		if (d != axis) {
			ax[n] = d;
			ext[n] = g.sizes[d];
			n++;
		}
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= (long long)ext[0] * ext[1]) return;
	const unsigned c = map[i];
	if (c == kNoFaceCond) return;
	long long base = g.origin + (long long)(side > 0 ? g.sizes[axis] - 1 : 0) * g.stride[axis];
	if (n == 1) base += i * g.stride[ax[0]];
	if (n == 2) base += (i / ext[1]) * g.stride[ax[0]] + (i % ext[1]) * g.stride[ax[1]];
	border_point(cur, g, base, axis, side > 0 ? -1 : 1, bq[c]);  // the table read in place
}

// A face map's condition tables into device memory, ordered on the stream (no
// host synchronisation; kernel-argument values read with uniform indices only).
__global__ __launch_bounds__(64) void k_set_face_tables(BorderQ* __restrict__ bq, FaceCond* __restrict__ fc,
                                                        FaceTables t) {
	if (threadIdx.x != 0) return;
	for (int k = 0; k < t.n; k++) {
		bq[k] = t.bq[k];
		fc[k] = t.fc[k];
	}
}

// ---------------------------------------------------------------- launchers --

template <int D, int BS>
static void launch_generic_dbs(const double* cur, double* nxt, const Geo& g, int s,
                               const AxisTable* tabs, const uint8_t* mat, hipStream_t st) {
	const long long blocks = (g.n_inner + 255) / 256;
	if (mat)
		hipLaunchKernelGGL((k_stage_generic<D, BS, true>), dim3((unsigned)blocks), dim3(256), 0,
		                   st, cur, nxt, g, s, tabs, mat);
	else
		hipLaunchKernelGGL((k_stage_generic<D, BS, false>), dim3((unsigned)blocks), dim3(256),
		                   0, st, cur, nxt, g, s, tabs, mat);
}

template <int D>
static bool launch_generic_d(const double* cur, double* nxt, const Geo& g, int s,
                             const AxisTable* tabs, const uint8_t* mat, hipStream_t st) {
	switch (g.bs) {
	case 1: launch_generic_dbs<D, 1>(cur, nxt, g, s, tabs, mat, st); return true;
	case 2: launch_generic_dbs<D, 2>(cur, nxt, g, s, tabs, mat, st); return true;
	case 3: launch_generic_dbs<D, 3>(cur, nxt, g, s, tabs, mat, st); return true;
	case 4: launch_generic_dbs<D, 4>(cur, nxt, g, s, tabs, mat, st); return true;
	case 5: launch_generic_dbs<D, 5>(cur, nxt, g, s, tabs, mat, st); return true;
	case 6: launch_generic_dbs<D, 6>(cur, nxt, g, s, tabs, mat, st); return true;
	case 7: launch_generic_dbs<D, 7>(cur, nxt, g, s, tabs, mat, st); return true;
	case 8: launch_generic_dbs<D, 8>(cur, nxt, g, s, tabs, mat, st); return true;
	default: return false;
	}
}

bool launch_stage_generic(const double* cur, double* nxt, const Geo& g, int s,
                          const AxisTable* tabs, const uint8_t* mat, hipStream_t st) {
	switch (g.D) {
	case 1: return launch_generic_d<1>(cur, nxt, g, s, tabs, mat, st);
	case 2: return launch_generic_d<2>(cur, nxt, g, s, tabs, mat, st);
	case 3: return launch_generic_d<3>(cur, nxt, g, s, tabs, mat, st);
	default: return false;
	}
}

void launch_fill_random(double* cur, const Geo& g, const int gstart[3], long long GY,
                        long long GZ, uint64_t seed, hipStream_t st) {
	const long long blocks = (g.n_inner + 255) / 256;
	hipLaunchKernelGGL(k_fill_random, dim3((unsigned)blocks), dim3(256), 0, st, cur, g,
	                   gstart[0], gstart[1], gstart[2], GY, GZ, seed);
}

void launch_copy_box(double* dst, const Geo& gd, const double* src, const Geo& gs,
                     const int dmin[3], const int smin[3], const int ext[3], hipStream_t st) {
	const long long n = (long long)ext[0] * ext[1] * ext[2];
	if (n <= 0) return;
	hipLaunchKernelGGL(k_copy_box, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, gd,
	                   src, gs, dmin[0], dmin[1], dmin[2], smin[0], smin[1], smin[2], ext[0],
	                   ext[1], ext[2]);
}

// MaxwellViscosityOde::apply (rheology/ode/Ode.hpp:28-37): every stress
// component of every inner node times exp(-tau / tau0) of the node's material
// (the factor per material is computed on the host, once, like the reference
// computes it per node: same libm call, same bits).  One thread per inner node.
__global__ __launch_bounds__(256) void k_scale_stress(double* __restrict__ cur, Geo g,
                                                      const uint8_t* __restrict__ mat,
                                                      const double* __restrict__ f_d, double f0) {
	const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= g.n_inner) return;
	const int z = (int)(i % g.sizes[2]);
	const long long t = i / g.sizes[2];
	const int y = (int)(t % g.sizes[1]);
	const int x = (int)(t / g.sizes[1]);
	const long long off = g.origin + x * g.stride[0] + y * g.stride[1] + z * g.stride[2];
	const double f = mat ? f_d[mat[i]] : f0;
	for (int c = g.D; c < g.M; c++) cur[c * g.cs + off] = cur[c * g.cs + off] * f;
}

// The per-material factors into device memory, ordered on the stream (no host
// synchronisation): kernel-argument values read with uniform indices only.
__global__ __launch_bounds__(64) void k_set_factors(double* __restrict__ dst, OdeFactors v) {
	if (threadIdx.x != 0) return;
	for (int m = 0; m < v.n; m++) dst[m] = v.f[m];
}

void launch_set_factors(double* dst_d, const OdeFactors& v, hipStream_t st) {
	hipLaunchKernelGGL(k_set_factors, dim3(1), dim3(64), 0, st, dst_d, v);
}

void launch_scale_stress(double* cur, const Geo& g, const uint8_t* mat_d, const double* f_d,
                         double f0, hipStream_t st) {
	if (g.n_inner <= 0) return;
	hipLaunchKernelGGL(k_scale_stress, dim3((unsigned)((g.n_inner + 255) / 256)), dim3(256), 0, st,
	                   cur, g, mat_d, f_d, f0);
}

void launch_border_fill(double* cur, const Geo& g, int axis, int inner_sign, int n_nodes,
                        const int* nodes_d, const BorderQ& bq, hipStream_t st) {
	if (n_nodes <= 0) return;
	hipLaunchKernelGGL(k_border_fill, dim3((n_nodes + 63) / 64), dim3(64), 0, st, cur, g, axis,
	                   inner_sign, n_nodes, nodes_d, bq);
}

void launch_face_fill(double* cur, const Geo& g, int axis, int side, const BorderQ& bq,
                      hipStream_t st) {
	long long n = 1;
	for (int d = 0; d < g.D; d++)
		if (d != axis) n *= g.sizes[d];
	const dim3 grid((unsigned)((n + 255) / 256));
	if (g.D == 3 && g.M == 9) {
		FaceCond fc{};
		bool plain = true;
		for (int k = 0; k < bq.n && plain; k++) {
			const int c = quantity_component(3, bq.q[k]);
			if (bq.q[k] == 12) plain = false;  // PRESSURE: the generic form
			if (c < 0) continue;
			fc.mask |= 1u << c;
			fc.two_v[c] = 2 * bq.v[k];
		}
		if (plain) {
			hipLaunchKernelGGL(k_face_fill9, dim3(grid.x, 9), dim3(256), 0, st, cur, g, axis, side, fc);
			return;
		}
	}
	hipLaunchKernelGGL(k_face_fill, grid, dim3(256), 0, st, cur, g, axis, side, bq);
}

void launch_face_fill_map(double* cur, const Geo& g, int axis, int side, const uint8_t* map_d,
                          const BorderQ* bq_d, hipStream_t st) {
	long long n = 1;
	for (int d = 0; d < g.D; d++)
		if (d != axis) n *= g.sizes[d];
	hipLaunchKernelGGL(k_face_fill_map, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cur, g, axis, side,
	                   map_d, bq_d);
}

void launch_set_face_tables(BorderQ* bq_d, FaceCond* fc_d, const FaceTables& t, hipStream_t st) {
	hipLaunchKernelGGL(k_set_face_tables, dim3(1), dim3(64), 0, st, bq_d, fc_d, t);
}

}  // namespace gcmx
