// kernels_fast.hip -- 3-D isotropic-elastic stage kernels for gfx950.
//
// Same arithmetic as k_stage_generic (and therefore as the reference stage,
// engine/cubic/GridCharacteristicMethod.hpp:42-52), specialised at compile time
// on the zero pattern of the isotropic-elastic U / U1 in the axis-aligned basis
// (ElasticModel.hpp:416-553) and on the eigenvalue structure
// L = (c1,-c1,c2,-c2,c2,-c2,0,0,0) (ElasticModel.hpp:401-407).  The host checks
// that the actual matrices fit the pattern before choosing these kernels.
//
//   k_march<S>   : stage along a strided axis S in {0 (X), 1 (Y)}.  One thread per
//                  (other axis, z) column marches along S keeping a register
//                  window of 2*BS+1 planes, so every element is read from HBM
//                  once (plus a 2*BS-plane halo per chunk).
//   k_line_z     : stage along the contiguous axis Z: a 256-node row segment plus
//                  its BS-node halos staged in LDS, neighbours read from LDS.
//   k_fused_yz   : Y stage then Z stage of one time step in ONE pass.  A block owns
//                  one x plane and a chunk of y rows with the whole z row; it
//                  marches along y (register window), hands each Y-stage row to
//                  the Z stage through LDS and writes only the Z-stage result.
//                  Halves the HBM traffic of the Y/Z stages.
#include "common.hpp"
#include "launch.hpp"

namespace gcmx {

// --------------------------------------------------------- zero patterns --

// Index of sigma(i,j) in the 3-D PDE vector (VelocitySigmaVariables.hpp:82-96).
__host__ __device__ constexpr int sig3(int i, int j) {
	return (i <= j) ? 3 + (i * 3 - ((i - 1) * i) / 2 + j - i)
	                : 3 + (j * 3 - ((j - 1) * j) / 2 + i - j);
}
__host__ __device__ constexpr unsigned bit(int i) { return 1u << i; }

// Tangent axes of createLocalBasis(e_s) (linal/basis.hpp:58-65).
__host__ __device__ constexpr int tang1(int s) { return s == 0 ? 1 : 0; }
__host__ __device__ constexpr int tang2(int s) { return s == 2 ? 1 : 2; }

// Non-zero columns of row k of U (ElasticModel.hpp:486-553).
__host__ __device__ constexpr unsigned iso_u_row(int s, int k) {
	const int t1 = tang1(s), t2 = tang2(s);
	return (k < 2)   ? (bit(s) | bit(sig3(s, s)))
	       : (k < 4) ? (bit(t1) | bit(sig3(t1, s)))
	       : (k < 6) ? (bit(t2) | bit(sig3(t2, s)))
	       : (k == 6) ? bit(sig3(t1, t2))
	       : (k == 7) ? (bit(sig3(t1, t1)) | bit(sig3(t2, t2)))
	                  : (bit(sig3(t1, t1)) | bit(sig3(t2, t2)) | bit(sig3(s, s)));
}
// Non-zero rows of column n of U1 (ElasticModel.hpp:416-483).
__host__ __device__ constexpr unsigned iso_u1_col(int s, int n) {
	const int t1 = tang1(s), t2 = tang2(s);
	return (n < 2)   ? (bit(s) | bit(sig3(0, 0)) | bit(sig3(1, 1)) | bit(sig3(2, 2)))
	       : (n < 4) ? (bit(t1) | bit(sig3(s, t1)))
	       : (n < 6) ? (bit(t2) | bit(sig3(s, t2)))
	       : (n == 6) ? bit(sig3(t1, t2))
	                  : (bit(sig3(t1, t1)) | bit(sig3(t2, t2)));
}
__host__ __device__ constexpr bool iso_u1(int s, int c, int n) {
	return (iso_u1_col(s, n) >> c) & 1u;
}
__host__ __device__ constexpr bool iso_u(int s, int k, int j) {
	return (iso_u_row(s, k) >> j) & 1u;
}
// Components read at the neighbours (rows with non-zero eigenvalue).
__host__ __device__ constexpr unsigned iso_window(int s) {
	return iso_u_row(s, 0) | iso_u_row(s, 2) | iso_u_row(s, 4);
}
// Components read only at the node itself.
__host__ __device__ constexpr unsigned iso_center_only(int s) {
	return (iso_u_row(s, 6) | iso_u_row(s, 7) | iso_u_row(s, 8)) & ~iso_window(s);
}
// Position of component j among the window components.
__host__ __device__ constexpr int wslot(unsigned mask, int j) {
	int n = 0;
	for (int i = 0; i < j; i++) n += (mask >> i) & 1u;
	return n;
}
__host__ __device__ constexpr int popc9(unsigned m) {
	int n = 0;
	for (int i = 0; i < 9; i++) n += (m >> i) & 1u;
	return n;
}

bool iso_pattern_fits(int s, const double* U, const double* U1, const double* L) {
	for (int k = 0; k < 9; k++) {
		if (k < 6) {
			if (!((k % 2 == 0) ? (L[k] > 0) : (L[k] < 0))) return false;
		} else if (L[k] != 0.0) {
			return false;
		}
		for (int j = 0; j < 9; j++) {
			if (U[k * 9 + j] != 0.0 && !iso_u(s, k, j)) return false;
			if (U1[k * 9 + j] != 0.0 && !iso_u1(s, k, j)) return false;
		}
	}
	return true;
}

// Reads of the uniform per-axis table.  The table sits in global memory; every
// index is a compile-time constant, so these are scalar loads through the
// scalar cache (s_load), never VGPR traffic.
struct Tab {
	const AxisTable* __restrict__ t;
	__device__ __forceinline__ double u(int k, int j) const { return t->U[k * 9 + j]; }
	__device__ __forceinline__ double u1(int c, int n) const { return t->U1[c * 9 + n]; }
	__device__ __forceinline__ int kf(int k) const { return t->kf[k]; }
	__device__ __forceinline__ const double* coef(int k) const { return t->coef[k]; }
};

// One node's stage given accessor functors:
//   W(j, o) = value of window component j at offset o (|o| <= BS) along S,
//   C(j)    = value of component j at the node (any component the rows 6..8 use).
// Returns the 9 outputs.  Operation order = reference (see kernels_generic.hip).
template <int S, int BS, class WF, class CF>
__device__ __forceinline__ void node_update(const Tab& T, WF W, CF C, double (&out)[9]) {
	double r[9];
#pragma unroll
	for (int k = 0; k < 9; k++) {
		double acc = 0.0;
		bool first = true;
#pragma unroll
		for (int j = 0; j < 9; j++) {
			if (!iso_u(S, k, j)) continue;
			double v;
			if (k < 6) {
				double sv[BS + 1];
				const int sh = (k % 2 == 0) ? -1 : 1;  // L>0 -> dx<0 -> shift -1
#pragma unroll
				for (int a = 0; a <= BS; a++) sv[a] = W(j, sh * a);
				v = newton_minmax<BS>(sv, T.kf(k), T.coef(k));
			} else {
				v = C(j);  // q == 0: the interpolant is the node value
			}
			const double u = T.u(k, j);
			acc = first ? u * v : acc + u * v;
			first = false;
		}
		r[k] = acc;
	}
#pragma unroll
	for (int c = 0; c < 9; c++) {
		double acc = 0.0;
		bool first = true;
#pragma unroll
		for (int n = 0; n < 9; n++) {
			if (!iso_u1(S, c, n)) continue;
			const double w = T.u1(c, n);
			acc = first ? w * r[n] : acc + w * r[n];
			first = false;
		}
		out[c] = acc;
	}
}

// ---------------------------------------------------------------- march --

constexpr int kMarchThreads = 256;

// Stage along S (0 = X, 1 = Y) for planes [m0, m1) of axis S in chunks of
// `chunk` planes; threads over (a, z), a = the other strided axis.
template <int S, int BS>
__global__ __launch_bounds__(kMarchThreads) void k_march(const double* __restrict__ cur,
                                                         double* __restrict__ nxt, Geo g,
                                                         const AxisTable* __restrict__ tab,
                                                         int m0, int m1, int chunk) {
	constexpr unsigned WM = iso_window(S);
	constexpr unsigned CM = iso_center_only(S);
	constexpr int NW = popc9(WM);
	constexpr int W = 2 * BS + 1;
	constexpr int A = 1 - S;  // the other strided axis
	const Tab T{tab};

	const int z = blockIdx.x * kMarchThreads + threadIdx.x;
	const int a = blockIdx.y;
	const int mb = m0 + blockIdx.z * chunk;
	const int me = min(mb + chunk, m1);
	if (z >= g.sizes[2]) return;
	const long long st = g.stride[S];
	const double* src = cur + g.origin + a * g.stride[A] + z;
	double* dst = nxt + g.origin + a * g.stride[A] + z;

	double win[NW][W];
	double ctr[9];
	// prologue: planes mb-BS .. mb+BS-1
#pragma unroll
	for (int j = 0; j < 9; j++) {
		if (!((WM >> j) & 1u)) continue;
#pragma unroll
		for (int o = 0; o < W - 1; o++)
			win[wslot(WM, j)][o] = src[j * g.cs + (long long)(mb - BS + o) * st];
	}
	// prefetch registers for the first iteration
	double pw[NW];
	double pc[9];
#pragma unroll
	for (int j = 0; j < 9; j++) {
		if ((WM >> j) & 1u) pw[wslot(WM, j)] = src[j * g.cs + (long long)(mb + BS) * st];
		if ((CM >> j) & 1u) pc[j] = src[j * g.cs + (long long)mb * st];
	}
	for (int m = mb; m < me; m++) {
#pragma unroll
		for (int j = 0; j < 9; j++) {
			if ((WM >> j) & 1u) win[wslot(WM, j)][W - 1] = pw[wslot(WM, j)];
			if ((CM >> j) & 1u) ctr[j] = pc[j];
		}
		if (m + 1 < me) {  // issue next iteration's loads before computing
#pragma unroll
			for (int j = 0; j < 9; j++) {
				if ((WM >> j) & 1u)
					pw[wslot(WM, j)] = src[j * g.cs + (long long)(m + 1 + BS) * st];
				if ((CM >> j) & 1u) pc[j] = src[j * g.cs + (long long)(m + 1) * st];
			}
		}
		double out[9];
		node_update<S, BS>(
		    T, [&](int j, int o) { return win[wslot(WM, j)][BS + o]; },
		    [&](int j) { return ((WM >> j) & 1u) ? win[wslot(WM, j)][BS] : ctr[j]; }, out);
#pragma unroll
		for (int c = 0; c < 9; c++) dst[c * g.cs + (long long)m * st] = out[c];
#pragma unroll
		for (int q = 0; q < NW; q++)
#pragma unroll
			for (int o = 0; o < W - 1; o++) win[q][o] = win[q][o + 1];
	}
}

// --------------------------------------------------------------- line z --

constexpr int kLineThreads = 256;

template <int BS>
__global__ __launch_bounds__(kLineThreads) void k_line_z(const double* __restrict__ cur,
                                                         double* __restrict__ nxt, Geo g,
                                                         const AxisTable* __restrict__ tab,
                                                         int x0) {
	constexpr int S = 2;
	constexpr unsigned WM = iso_window(S);
	constexpr unsigned CM = iso_center_only(S);
	constexpr int NW = popc9(WM);
	constexpr int LW = kLineThreads + 2 * BS;
	__shared__ double lds[NW][LW];
	const Tab T{tab};

	const int z0 = blockIdx.x * kLineThreads;
	const int y = blockIdx.y;
	const int x = x0 + blockIdx.z;
	const int tid = threadIdx.x;
	const int Z = g.sizes[2];
	const long long rowoff = g.origin + x * g.stride[0] + y * g.stride[1];
	const double* src = cur + rowoff;
	// stage the row segment [z0-BS, z0+256+BS) of the window components
	for (int i = tid; i < LW; i += kLineThreads) {
		const int zz = z0 - BS + i;
		if (zz < Z + BS) {
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((WM >> j) & 1u) lds[wslot(WM, j)][i] = src[j * g.cs + zz];
		}
	}
	const int z = z0 + tid;
	double ctr[9];
#pragma unroll
	for (int j = 0; j < 9; j++)
		if (((CM >> j) & 1u) && z < Z) ctr[j] = src[j * g.cs + z];
	__syncthreads();
	if (z >= Z) return;
	double out[9];
	node_update<S, BS>(
	    T, [&](int j, int o) { return lds[wslot(WM, j)][BS + tid + o]; },
	    [&](int j) { return ((WM >> j) & 1u) ? lds[wslot(WM, j)][BS + tid] : ctr[j]; }, out);
	double* dst = nxt + rowoff + z;
#pragma unroll
	for (int c = 0; c < 9; c++) dst[c * g.cs] = out[c];
}

// -------------------------------------------------------------- fused yz --

// Block = one x plane, rows [yb, ye) of a y chunk, all z (blockDim = ZT >= Z).
// Reads the X-stage output `in` (Y-stage input), writes the Z-stage output to
// `out`.  `in` and `out` are different layers; the z-ghosts the Z stage reads
// are those of `out` (the layer the Y stage would have written).
template <int BS, int ZT>
__global__ __launch_bounds__(ZT) void k_fused_yz(const double* __restrict__ in,
                                                 double* __restrict__ outl, Geo g,
                                                 const AxisTable* __restrict__ tabY,
                                                 const AxisTable* __restrict__ tabZ, int x0,
                                                 int chunk) {
	constexpr unsigned WMY = iso_window(1);
	constexpr unsigned CMY = iso_center_only(1);
	constexpr int NWY = popc9(WMY);
	constexpr unsigned WMZ = iso_window(2);
	constexpr int NWZ = popc9(WMZ);
	constexpr int W = 2 * BS + 1;
	constexpr int LW = ZT + 2 * BS;
	__shared__ double lds[2][NWZ][LW];
	const Tab TY{tabY}, TZ{tabZ};

	const int z = threadIdx.x;
	const int x = x0 + blockIdx.y;
	const int Y = g.sizes[1], Z = g.sizes[2];
	const int yb = blockIdx.x * chunk;
	const int ye = min(yb + chunk, Y);
	const bool live = z < Z;
	const int zc = live ? z : Z - 1;  // clamp idle lanes onto a valid column
	const long long st = g.stride[1];
	const long long plane = g.origin + x * g.stride[0];
	const double* src = in + plane + zc;

	// z-ghost entries of the Z stage: 2*BS per row, loaded by threads [0, 2BS)
	const bool ghost_lane = z < 2 * BS;
	const int gz = (z < BS) ? (z - BS) : (Z + z - BS);  // ghost z index
	const int gslot = (z < BS) ? z : (Z + z);           // its LDS slot

	double win[NWY][W];
	double ctr[9];
#pragma unroll
	for (int j = 0; j < 9; j++) {
		if (!((WMY >> j) & 1u)) continue;
#pragma unroll
		for (int o = 0; o < W - 1; o++)
			win[wslot(WMY, j)][o] = src[j * g.cs + (long long)(yb - BS + o) * st];
	}
	double pw[NWY];
	double pc[9];
#pragma unroll
	for (int j = 0; j < 9; j++) {
		if ((WMY >> j) & 1u) pw[wslot(WMY, j)] = src[j * g.cs + (long long)(yb + BS) * st];
		if ((CMY >> j) & 1u) pc[j] = src[j * g.cs + (long long)yb * st];
	}
	int buf = 0;
	for (int y = yb; y < ye; y++) {
#pragma unroll
		for (int j = 0; j < 9; j++) {
			if ((WMY >> j) & 1u) win[wslot(WMY, j)][W - 1] = pw[wslot(WMY, j)];
			if ((CMY >> j) & 1u) ctr[j] = pc[j];
		}
		if (y + 1 < ye) {
#pragma unroll
			for (int j = 0; j < 9; j++) {
				if ((WMY >> j) & 1u)
					pw[wslot(WMY, j)] = src[j * g.cs + (long long)(y + 1 + BS) * st];
				if ((CMY >> j) & 1u) pc[j] = src[j * g.cs + (long long)(y + 1) * st];
			}
		}
		// ---- Y stage at (x, y, z)
		double yv[9];
		node_update<1, BS>(
		    TY, [&](int j, int o) { return win[wslot(WMY, j)][BS + o]; },
		    [&](int j) { return ((WMY >> j) & 1u) ? win[wslot(WMY, j)][BS] : ctr[j]; }, yv);
		// ---- hand the row to the Z stage
		const long long rowoff = plane + (long long)y * st;
		if (live) {
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((WMZ >> j) & 1u) lds[buf][wslot(WMZ, j)][BS + z] = yv[j];
		}
		if (ghost_lane) {
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((WMZ >> j) & 1u) lds[buf][wslot(WMZ, j)][gslot] = outl[rowoff + j * g.cs + gz];
		}
		__syncthreads();
		if (live) {
			double zv[9];
			node_update<2, BS>(
			    TZ, [&](int j, int o) { return lds[buf][wslot(WMZ, j)][BS + z + o]; },
			    [&](int j) { return ((WMZ >> j) & 1u) ? lds[buf][wslot(WMZ, j)][BS + z] : yv[j]; },
			    zv);
			double* dst = outl + rowoff + z;
#pragma unroll
			for (int c = 0; c < 9; c++) dst[c * g.cs] = zv[c];
		}
		buf ^= 1;
#pragma unroll
		for (int q = 0; q < NWY; q++)
#pragma unroll
			for (int o = 0; o < W - 1; o++) win[q][o] = win[q][o + 1];
	}
}

// ------------------------------------------------------------- launchers --

static int march_chunk(int len) { return len < 128 ? len : 64; }

template <int BS>
static void launch_march_bs(const double* cur, double* nxt, const Geo& g, int s,
                            const AxisTable* tab, int x0, int x1, hipStream_t st) {
	// For S = 0 the march axis is X ([x0,x1)); for S = 1 threads cover x in [x0,x1).
	if (s == 0) {
		const int len = x1 - x0;
		const int chunk = march_chunk(len);
		dim3 grid((g.sizes[2] + kMarchThreads - 1) / kMarchThreads, g.sizes[1],
		          (len + chunk - 1) / chunk);
		hipLaunchKernelGGL((k_march<0, BS>), grid, dim3(kMarchThreads), 0, st, cur, nxt, g, tab,
		                   x0, x1, chunk);
	} else {
		const int len = g.sizes[1];
		const int chunk = march_chunk(len);
		Geo gg = g;
		gg.origin = g.origin + (long long)x0 * g.stride[0];
		dim3 grid((g.sizes[2] + kMarchThreads - 1) / kMarchThreads, x1 - x0,
		          (len + chunk - 1) / chunk);
		hipLaunchKernelGGL((k_march<1, BS>), grid, dim3(kMarchThreads), 0, st, cur, nxt, gg,
		                   tab, 0, len, chunk);
	}
}

bool launch_march(const double* cur, double* nxt, const Geo& g, int s, const AxisTable* tab,
                  int x0, int x1, hipStream_t st) {
	if (g.D != 3 || s > 1 || x1 <= x0) return false;
	switch (g.bs) {
	case 1: launch_march_bs<1>(cur, nxt, g, s, tab, x0, x1, st); return true;
	case 2: launch_march_bs<2>(cur, nxt, g, s, tab, x0, x1, st); return true;
	case 3: launch_march_bs<3>(cur, nxt, g, s, tab, x0, x1, st); return true;
	default: return false;
	}
}

template <int BS>
static void launch_line_bs(const double* cur, double* nxt, const Geo& g, const AxisTable* tab,
                           int x0, int x1, hipStream_t st) {
	dim3 grid((g.sizes[2] + kLineThreads - 1) / kLineThreads, g.sizes[1], x1 - x0);
	hipLaunchKernelGGL((k_line_z<BS>), grid, dim3(kLineThreads), 0, st, cur, nxt, g, tab, x0);
}

bool launch_line_z(const double* cur, double* nxt, const Geo& g, const AxisTable* tab, int x0,
                   int x1, hipStream_t st) {
	if (g.D != 3 || x1 <= x0) return false;
	switch (g.bs) {
	case 1: launch_line_bs<1>(cur, nxt, g, tab, x0, x1, st); return true;
	case 2: launch_line_bs<2>(cur, nxt, g, tab, x0, x1, st); return true;
	case 3: launch_line_bs<3>(cur, nxt, g, tab, x0, x1, st); return true;
	default: return false;
	}
}

bool fused_yz_supported(const Geo& g) {
	return g.D == 3 && g.bs >= 1 && g.bs <= 3 && g.sizes[2] <= 1024 && g.sizes[2] >= 2 * g.bs;
}

static int fused_chunk(int Y) { return Y <= 64 ? Y : 64; }

template <int BS, int ZT>
static void launch_fused_t(const double* in, double* out, const Geo& g, const AxisTable* ty,
                           const AxisTable* tz, int x0, int x1, hipStream_t st) {
	const int chunk = fused_chunk(g.sizes[1]);
	dim3 grid((g.sizes[1] + chunk - 1) / chunk, x1 - x0);
	hipLaunchKernelGGL((k_fused_yz<BS, ZT>), grid, dim3(ZT), 0, st, in, out, g, ty, tz, x0,
	                   chunk);
}

template <int BS>
static bool launch_fused_bs(const double* in, double* out, const Geo& g, const AxisTable* ty,
                            const AxisTable* tz, int x0, int x1, hipStream_t st) {
	const int Z = g.sizes[2];
	if (Z <= 64) launch_fused_t<BS, 64>(in, out, g, ty, tz, x0, x1, st);
	else if (Z <= 128) launch_fused_t<BS, 128>(in, out, g, ty, tz, x0, x1, st);
	else if (Z <= 256) launch_fused_t<BS, 256>(in, out, g, ty, tz, x0, x1, st);
	else if (Z <= 512) launch_fused_t<BS, 512>(in, out, g, ty, tz, x0, x1, st);
	else launch_fused_t<BS, 1024>(in, out, g, ty, tz, x0, x1, st);
	return true;
}

bool launch_fused_yz(const double* in, double* out, const Geo& g, const AxisTable* ty,
                     const AxisTable* tz, int x0, int x1, hipStream_t st) {
	if (!fused_yz_supported(g) || x1 <= x0) return false;
	switch (g.bs) {
	case 1: return launch_fused_bs<1>(in, out, g, ty, tz, x0, x1, st);
	case 2: return launch_fused_bs<2>(in, out, g, ty, tz, x0, x1, st);
	case 3: return launch_fused_bs<3>(in, out, g, ty, tz, x0, x1, st);
	default: return false;
	}
}

}  // namespace gcmx
