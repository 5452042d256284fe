// kernels_2d.hip -- the one-pass 2-D time step for gfx950 (X then Y stage of
// cubic::Engine::nextTimeStep, Engine.cpp:90-121, in one kernel).
//
// Two kernels, both with the reference stage's arithmetic
// (GridCharacteristicMethod.hpp:42-52; this file is built with
// -ffp-contract=off, so a step is bitwise the two per-stage passes):
//   k_step2d_iso : the 2-D isotropic-elastic structure (ElasticModel<2>,
//                  ElasticModel.hpp:416-553) compiled in, like the 3-D kernels
//                  (iso.hpp): the host verifies U / U1 / L against it bitwise
//                  (iso2_axis_extract); borderSize <= 3;
//   k_step2d     : any matrices of one material through the per-axis tables
//                  (k_stage_generic's form), borderSize <= 5.
#include "iso.hpp"

#include <string>

namespace gcmx {

// ----------------------------------------------------------- structure --

// The 2-D PDE vector (VelocitySigmaVariables<2>): v0, v1, s00, s01, s11.
__host__ __device__ constexpr int sig2(int i, int j) {
	return (i <= j) ? 2 + (i * 2 - ((i - 1) * i) / 2 + j - i) : 2 + (j * 2 - ((j - 1) * j) / 2 + i - j);
}
// createLocalBasis(e_s) in 2-D (linal/basis.hpp): the tangent is sign * e_t.
__host__ __device__ constexpr int tang2d(int s) { return 1 - s; }
__host__ __device__ constexpr int sgn2d(int s) { return s == 0 ? -1 : 1; }

// U(k, j) of ElasticModel<2> along axis S: rows 0/1 the +-c1 pair, rows 2/3 the
// +-c2 pair, row 4 the zero eigenvalue (sigma_tt + g sigma_SS).
__host__ __device__ constexpr Coef iso2_u(int S, int k, int j) {
	const int t = tang2d(S), s1 = sgn2d(S);
	const int ss = sig2(S, S), st = sig2(t, S), tt = sig2(t, t);
	return (k == 0) ? (j == S ? Coef{kOne, 1} : j == ss ? Coef{kA, 1} : cz())
	     : (k == 1) ? (j == S ? Coef{kOne, 1} : j == ss ? Coef{kA, -1} : cz())
	     : (k == 2) ? (j == t ? Coef{kOne, s1} : j == st ? Coef{kB, s1} : cz())
	     : (k == 3) ? (j == t ? Coef{kOne, s1} : j == st ? Coef{kB, -s1} : cz())
	                : (j == tt ? Coef{kOne, 1} : j == ss ? Coef{kG, 1} : cz());
}
// U1(c, n): columns are the eigenvectors.
__host__ __device__ constexpr Coef iso2_u1(int S, int c, int n) {
	const int t = tang2d(S), s1 = sgn2d(S);
	const int ss = sig2(S, S), st = sig2(t, S), tt = sig2(t, t);
	return (n == 0) ? (c == S ? Coef{kHalf, 1} : c == ss ? Coef{kP1, 1} : c == tt ? Coef{kP2, 1} : cz())
	     : (n == 1) ? (c == S ? Coef{kHalf, 1} : c == ss ? Coef{kP1, -1} : c == tt ? Coef{kP2, -1} : cz())
	     : (n == 2) ? (c == t ? Coef{kHalf, s1} : c == st ? Coef{kS, s1} : cz())
	     : (n == 3) ? (c == t ? Coef{kHalf, s1} : c == st ? Coef{kS, -s1} : cz())
	                : (c == tt ? Coef{kOne, 1} : cz());
}
// Components read at the neighbours (rows 0..3) / only at the node (row 4).
__host__ __device__ constexpr unsigned iso2_window(int S) {
	unsigned m = 0;
	for (int k = 0; k < 4; k++)
		for (int j = 0; j < 5; j++)
			if (iso2_u(S, k, j).slot != kZero) m |= bit(j);
	return m;
}
__host__ __device__ constexpr unsigned iso2_center_only(int S) {
	unsigned m = 0;
	for (int j = 0; j < 5; j++)
		if (iso2_u(S, 4, j).slot != kZero) m |= bit(j);
	return m & ~iso2_window(S);
}

static double slot_value2(const IsoAxis& A, int slot) {
	switch (slot) {
	case kOne: return 1.0;
	case kHalf: return 0.5;
	case kA: return A.a;
	case kB: return A.b;
	case kG: return A.g;
	case kP1: return A.p1;
	case kP2: return A.p2;
	case kS: return A.s;
	default: return 0.0;
	}
}

bool iso2_axis_extract(int S, const double* U, const double* U1, const double* L, IsoAxis& A) {
	const int t = tang2d(S), s1 = sgn2d(S);
	const int ss = sig2(S, S), st = sig2(t, S), tt = sig2(t, t);
	A.a = U[0 * 5 + ss];
	A.b = s1 * U[2 * 5 + st];
	A.g = U[4 * 5 + ss];
	A.p1 = U1[ss * 5 + 0];
	A.p2 = U1[tt * 5 + 0];
	A.s = s1 * U1[st * 5 + 2];
	for (int k = 0; k < 5; k++)
		for (int j = 0; j < 5; j++) {
			const Coef cu = iso2_u(S, k, j), cu1 = iso2_u1(S, k, j);
			if (!(U[k * 5 + j] == cu.sign * slot_value2(A, cu.slot)) ||
			    !(U1[k * 5 + j] == cu1.sign * slot_value2(A, cu1.slot)))
				return false;
			if (cu.slot == kZero && U[k * 5 + j] != 0.0) return false;
			if (cu1.slot == kZero && U1[k * 5 + j] != 0.0) return false;
		}
	// eigenvalues +-c1, +-c2, 0 with the pairs bitwise opposite
	return L[0] > 0 && L[1] == -L[0] && L[2] > 0 && L[3] == -L[2] && L[4] == 0.0;
}

// Unrolled sum over j of U(k, j) * V(j) (or U1(c, n) * r(n)) in ascending index
// order, structural zeros skipped, from the first non-zero term (iso.hpp RowSum).
template <int S, bool ISU1, int ROW, int J = 0>
struct RowSum2 {
	template <class F>
	__device__ __forceinline__ static double go(const IsoAxis& A, F val, double acc, bool first) {
		if constexpr (J == 5) {
			return acc;
		} else {
			constexpr Coef c = ISU1 ? iso2_u1(S, ROW, J) : iso2_u(S, ROW, J);
			if constexpr (c.slot == kZero) {
				return RowSum2<S, ISU1, ROW, J + 1>::go(A, val, acc, first);
			} else {
				const double t = term<c.slot, c.sign>(A, val(J));
				return RowSum2<S, ISU1, ROW, J + 1>::go(A, val, first ? t : acc + t, false);
			}
		}
	}
};

// One node's stage along S.  W(j, o): component j at offset o (|o| <= BS) for
// the window components; C(j): the node value of a component row 4 reads.
template <int S, int BS, bool KF0, class WF, class CF>
__device__ __forceinline__ void node_update2(const IsoAxis& A, WF W, CF C, double (&out)[5]) {
	double r[5];
	auto interp = [&](int j, int sh, const double* coef, int kf) {
		double sv[BS + 1];
#pragma unroll
		for (int i = 0; i <= BS; i++) sv[i] = W(j, sh * i);
		return newton_minmax<BS, KF0>(sv, kf, coef);
	};
	// rows 2P: foot on the -S side (L > 0); rows 2P+1: the +S side
	r[0] = RowSum2<S, false, 0>::go(A, [&](int j) { return interp(j, -1, A.c1, A.kf1); }, 0.0, true);
	r[1] = RowSum2<S, false, 1>::go(A, [&](int j) { return interp(j, 1, A.c1, A.kf1); }, 0.0, true);
	r[2] = RowSum2<S, false, 2>::go(A, [&](int j) { return interp(j, -1, A.c2, A.kf2); }, 0.0, true);
	r[3] = RowSum2<S, false, 3>::go(A, [&](int j) { return interp(j, 1, A.c2, A.kf2); }, 0.0, true);
	r[4] = RowSum2<S, false, 4>::go(A, C, 0.0, true);
	auto rv = [&](int n) { return r[n]; };
	out[0] = RowSum2<S, true, 0>::go(A, rv, 0.0, true);
	out[1] = RowSum2<S, true, 1>::go(A, rv, 0.0, true);
	out[2] = RowSum2<S, true, 2>::go(A, rv, 0.0, true);
	out[3] = RowSum2<S, true, 3>::go(A, rv, 0.0, true);
	out[4] = RowSum2<S, true, 4>::go(A, rv, 0.0, true);
}

// The one-pass 2-D step on the isotropic structure: the block / lane layout of
// k_step2d below (T lanes along y, T - 2*BS of them written, the march along x
// with a register window), with only the components the structure reads: the
// X stage reads four components at the neighbouring rows and sigma_yy at the
// node; the Y stage reads four X results at the neighbouring lanes (LDS) and
// sigma_xx at its own lane (a register).  Layer planes < 2^32 bytes (32-bit
// element offsets, step2d_iso_supported).
#ifndef GCMX_2D_PF  // rows the loads run ahead of the row computed
#define GCMX_2D_PF 1
#endif
//
// FACES: border conditions on the y faces (Face2).  A lane whose column is a
// ghost of a face with a condition loads the MIRRORED inner column (ghost -a <->
// inner +a, BorderConditions.hpp:94-114) and forms that column's X stage itself
// -- the same operations on the same data as the lane that owns it, so the same
// bits -- then stores the ghost value (the mirrored X result, -inner + 2 f(t) in
// the overridden components) in its LDS slot: the Y stage reads ghost columns
// like any other, with no extra barrier and no divergent branch.
template <int BS, int T, bool KF0, bool FACES>
__global__ __launch_bounds__(T) void k_step2d_iso(const double* __restrict__ cur, double* __restrict__ nxt, Geo g,
                                                  IsoAxis AX, IsoAxis AY, int chunk, Face2 fc) {
	constexpr unsigned WMX = iso2_window(0), CMX = iso2_center_only(0);
	constexpr unsigned WMY = iso2_window(1);
	constexpr int NWX = popc9(WMX), NWY = popc9(WMY);
	constexpr int W = 2 * BS + 1;
	constexpr int PD = GCMX_2D_PF;
	__shared__ double lds[2][NWY][T];
	const int l = threadIdx.x;
	const int X = g.sizes[0], Y = g.sizes[1];
	const int y = (int)blockIdx.x * (T - 2 * BS) - BS + l;
	const int xb = (int)blockIdx.y * chunk;
	const int xe = min(xb + chunk, X);
	const bool inner = y >= 0 && y < Y;
	const bool out = inner && l >= BS && l < T - BS;
	// FACES: a ghost column of a face with a condition forms its mirror's X stage
	const int face = y < 0 ? 0 : 1;
	const bool ghost = FACES && !inner && y >= -BS && y < Y + BS && ((fc.on >> face) & 1u);
	const int ysrc = inner ? y : ghost ? (y < 0 ? -y : 2 * (Y - 1) - y) : 0;
	const bool col = inner || ghost;  // the lane loads a column and forms its X stage
	const unsigned sx = (unsigned)g.stride[0];
	const unsigned off = (unsigned)(g.origin + ysrc);  // + x * sx: node (x, ysrc)
	const unsigned fmask = ghost ? fc.mask[face] : 0u;
	const Planes src(cur, g.cs);
	const PlanesW dst(nxt, g.cs);

	// win: rows x - BS .. x + BS of the window components, ctr: row x of the
	// node-only one; pw[d] / pc[d]: rows x + 1 + d + BS / x + 1 + d, in flight
	double win[NWX][W], pw[PD][NWX];
	double ctr[5], pc[PD][5];
	auto load_ahead = [&](int r, double (&w)[NWX], double (&c)[5]) {  // row r = x + 1 + d
		const bool ok = col && r < xe;
#pragma unroll
		for (int j = 0; j < 5; j++) {
			if ((WMX >> j) & 1u) w[wslot(WMX, j)] = ok ? src.ld(j, off + (unsigned)(r + BS) * sx) : 0.0;
			if ((CMX >> j) & 1u) c[j] = ok ? src.ld(j, off + (unsigned)r * sx) : 0.0;
		}
	};
#pragma unroll
	for (int j = 0; j < 5; j++) {
		if ((WMX >> j) & 1u) {
#pragma unroll
			for (int o = 0; o < W; o++)
				win[wslot(WMX, j)][o] = col ? src.ld(j, off + (unsigned)(xb - BS + o) * sx) : 0.0;
		}
		if ((CMX >> j) & 1u) ctr[j] = col ? src.ld(j, off + (unsigned)xb * sx) : 0.0;
	}
#pragma unroll
	for (int d = 0; d < PD - 1; d++) load_ahead(xb + 1 + d, pw[d], pc[d]);

	for (int x = xb; x < xe; x++) {
		load_ahead(x + PD, pw[PD - 1], pc[PD - 1]);
		double xo[5];
		node_update2<0, BS, KF0>(
		    AX, [&](int j, int o) { return win[wslot(WMX, j)][BS + o]; },
		    [&](int j) { return ((WMX >> j) & 1u) ? win[wslot(WMX, j)][BS] : ctr[j]; }, xo);
		double (*buf)[T] = lds[x & 1];
#pragma unroll
		for (int c = 0; c < 5; c++)
			if ((WMY >> c) & 1u) {
				double v = col ? xo[c] : 0.0;  // ghost columns without a condition: 0
				if constexpr (FACES)
					if ((fmask >> c) & 1u) v = -v + fc.two_v[face][c];
				buf[wslot(WMY, c)][l] = v;
			}
		__syncthreads();
		if (out) {
			double yo[5];
			node_update2<1, BS, KF0>(
			    AY, [&](int j, int o) { return buf[wslot(WMY, j)][l + o]; },
			    [&](int j) { return ((WMY >> j) & 1u) ? buf[wslot(WMY, j)][l] : xo[j]; }, yo);
			const unsigned o = off + (unsigned)x * sx;
#pragma unroll
			for (int c = 0; c < 5; c++) dst.st(c, o, yo[c]);  // non-temporal: 2.5 % slower
		}
#pragma unroll
		for (int q = 0; q < NWX; q++) {
#pragma unroll
			for (int o = 0; o < W - 1; o++) win[q][o] = win[q][o + 1];
			win[q][W - 1] = pw[0][q];
		}
#pragma unroll
		for (int j = 0; j < 5; j++)
			if ((CMX >> j) & 1u) ctr[j] = pc[0][j];
#pragma unroll
		for (int d = 0; d < PD - 1; d++) {
#pragma unroll
			for (int q = 0; q < NWX; q++) pw[d][q] = pw[d + 1][q];
#pragma unroll
			for (int j = 0; j < 5; j++) pc[d][j] = pc[d + 1][j];
		}
	}
}

// ------------------------------------------------------- table kernel --

// The whole 2-D time step in ONE pass through the per-axis tables: one
// material of any matrices, any borderSize up to 5, any Courant number.  The
// arithmetic of each stage is k_stage_generic's (the same skipped exact zeros,
// the same summation order), so the step is bitwise the two generic stages.
//
// Block = T lanes along the contiguous axis y and a chunk of x rows.  Lane l
// holds column y = y0 - BS + l: the block writes the T - 2*BS columns
// [y0, y0 + T - 2*BS) and computes the X stage of BS more columns on each side
// itself (the Y stage's halo), so no block reads another's intermediate.  Each
// thread marches x with a register window of the 2*BS+1 rows of every
// component (each element of the input layer read once per block, plus the
// 2*BS-row prologue), forms the X stage of its column at row x and hands it to
// the Y stage through double-buffered LDS: one barrier per row.
// HBM traffic: the input layer once, the output layer once (2*5*8 = 80 B per
// node-step instead of the two stage passes' 160).
// Preconditions (checked by the caller): every y ghost column of both layers
// is zero, so the X-stage results the Y stage reads at ghost columns are 0.0
// (the reference's stage writes inner nodes only, and nothing else wrote the
// ghosts); x ghost rows of `cur` hold what the X stage must read.
template <int BS, int T>
__global__ __launch_bounds__(T) void k_step2d(const double* __restrict__ cur, double* __restrict__ nxt, Geo g,
                                              const AxisTable* __restrict__ tabs, int chunk) {
	constexpr int M = 5;
	constexpr int W = 2 * BS + 1;
	__shared__ double lds[2][M][T];
	const int l = threadIdx.x;
	const int X = g.sizes[0], Y = g.sizes[1];
	const int y = (int)blockIdx.x * (T - 2 * BS) - BS + l;
	const int xb = (int)blockIdx.y * chunk;
	const int xe = min(xb + chunk, X);
	const bool col = y >= 0 && y < Y;                  // an inner column: its X stage is formed
	const bool out = col && l >= BS && l < T - BS;     // a column this block writes
	const long long sx = g.stride[0];
	const long long cs = g.cs;
	const long long base = g.origin + (col ? y : 0);  // + x * sx: node (x, y)
	const AxisTable& TX = tabs[0];
	const AxisTable& TY = tabs[1];

	double win[M][W];  // rows x - BS .. x + BS of every component
	double pf[M];      // row x + 1 + BS, in flight
#pragma unroll
	for (int j = 0; j < M; j++)
#pragma unroll
		for (int o = 0; o < W; o++)
			win[j][o] = col ? cur[j * cs + base + (long long)(xb - BS + o) * sx] : 0.0;

	for (int x = xb; x < xe; x++) {
		const bool more = x + 1 < xe;
#pragma unroll
		for (int j = 0; j < M; j++)
			pf[j] = (col && more) ? cur[j * cs + base + (long long)(x + 1 + BS) * sx] : 0.0;

		// X stage of (x, y): k_stage_generic with the neighbours from the window
		double r[M];
#pragma unroll
		for (int k = 0; k < M; k++) {
			const int sh = TX.shift[k];
			const int kf = TX.kf[k];
			const bool zq = TX.zero_q[k] != 0;
			double acc = 0.0;
			bool first = true;
#pragma unroll
			for (int j = 0; j < M; j++) {
				const double u = TX.U[k * M + j];
				if (u != 0.0) {
					double v;
					if (zq) {
						v = win[j][BS];
					} else {
						double sv[BS + 1];
						if (sh > 0) {
#pragma unroll
							for (int a = 0; a <= BS; a++) sv[a] = win[j][BS + a];
						} else {
#pragma unroll
							for (int a = 0; a <= BS; a++) sv[a] = win[j][BS - a];
						}
						v = newton_minmax<BS>(sv, kf, TX.coef[k]);
					}
					acc = first ? u * v : acc + u * v;
					first = false;
				}
			}
			r[k] = acc;
		}
		double (*buf)[T] = lds[x & 1];
#pragma unroll
		for (int c = 0; c < M; c++) {
			double acc = 0.0;
			bool first = true;
#pragma unroll
			for (int n = 0; n < M; n++) {
				const double w = TX.U1[c * M + n];
				if (w != 0.0) {
					acc = first ? w * r[n] : acc + w * r[n];
					first = false;
				}
			}
			buf[c][l] = col ? acc : 0.0;  // ghost columns: the zero the reference reads
		}
		__syncthreads();

		if (out) {  // Y stage of (x, y) from the X results of the neighbouring lanes
#pragma unroll
			for (int k = 0; k < M; k++) {
				const int sh = TY.shift[k];
				const int kf = TY.kf[k];
				const bool zq = TY.zero_q[k] != 0;
				double acc = 0.0;
				bool first = true;
#pragma unroll
				for (int j = 0; j < M; j++) {
					const double u = TY.U[k * M + j];
					if (u != 0.0) {
						double v;
						if (zq) {
							v = buf[j][l];
						} else {
							double sv[BS + 1];
#pragma unroll
							for (int a = 0; a <= BS; a++) sv[a] = buf[j][l + a * sh];
							v = newton_minmax<BS>(sv, kf, TY.coef[k]);
						}
						acc = first ? u * v : acc + u * v;
						first = false;
					}
				}
				r[k] = acc;
			}
			const long long o = base + (long long)x * sx;
#pragma unroll
			for (int c = 0; c < M; c++) {
				double acc = 0.0;
				bool first = true;
#pragma unroll
				for (int n = 0; n < M; n++) {
					const double w = TY.U1[c * M + n];
					if (w != 0.0) {
						acc = first ? w * r[n] : acc + w * r[n];
						first = false;
					}
				}
				nxt[c * cs + o] = acc;
			}
		}
#pragma unroll
		for (int j = 0; j < M; j++) {
#pragma unroll
			for (int o = 0; o < W - 1; o++) win[j][o] = win[j][o + 1];
			win[j][W - 1] = pf[j];
		}
	}
}

// ------------------------------------------------------------ launchers --

// rows per block: up to 64, fewer while the grid has under 1 024 blocks (the
// prologue costs 2*BS row loads, mostly cache hits)
static int step2d_chunk(int X, int ny) {
	int chunk = X < 64 ? X : 64;
	while (chunk > 4 && (long long)ny * ((X + chunk - 1) / chunk) < 1024) chunk = (chunk + 1) / 2;
	// gridDim.y <= 65535: beyond ~4.19M x rows a block marches more rows (any chunk is valid)
	while ((X + chunk - 1) / chunk > 65535) chunk *= 2;
	return chunk;
}

template <int BS, int T, bool KF0, bool FACES>
static const char* step2d_iso_name() {
	static const std::string s = "k_step2d_iso<" + std::to_string(BS) + ", " + std::to_string(T) + ", " +
	                             (KF0 ? "KF0" : "!KF0") + (FACES ? ", FACES" : "") + ">";
	return s.c_str();
}

template <int BS, int T>
static void launch_step2d_t(const double* cur, double* nxt, const Geo& g, const AxisTable* tabs,
                            const IsoAxis* iso, hipStream_t st, const char** kname, const Face2* faces) {
	const int X = g.sizes[0], Y = g.sizes[1];
	const int ny = (Y + (T - 2 * BS) - 1) / (T - 2 * BS);
	const int chunk = step2d_chunk(X, ny);
	const dim3 grid((unsigned)ny, (unsigned)((X + chunk - 1) / chunk));
	if constexpr (BS <= 3) {
		if (iso) {
			const bool kf0 = iso[0].kf1 == 0 && iso[0].kf2 == 0 && iso[1].kf1 == 0 && iso[1].kf2 == 0;
			const Face2 none{};
			auto go = [&](auto K, const char* name) {
				hipLaunchKernelGGL(K, grid, dim3(T), 0, st, cur, nxt, g, iso[0], iso[1], chunk, faces ? *faces : none);
				if (kname) *kname = name;
			};
			if (faces && faces->on) {
				if (kf0) go(k_step2d_iso<BS, T, true, true>, step2d_iso_name<BS, T, true, true>());
				else go(k_step2d_iso<BS, T, false, true>, step2d_iso_name<BS, T, false, true>());
			} else {
				if (kf0) go(k_step2d_iso<BS, T, true, false>, step2d_iso_name<BS, T, true, false>());
				else go(k_step2d_iso<BS, T, false, false>, step2d_iso_name<BS, T, false, false>());
			}
			return;
		}
	}
	hipLaunchKernelGGL((k_step2d<BS, T>), grid, dim3(T), 0, st, cur, nxt, g, tabs, chunk);
	static const std::string name = "k_step2d<" + std::to_string(BS) + ", " + std::to_string(T) + ">";
	if (kname) *kname = name.c_str();
}

template <int BS>
static void launch_step2d_bs(const double* cur, double* nxt, const Geo& g, const AxisTable* tabs,
                             const IsoAxis* iso, hipStream_t st, const char** kname, const Face2* faces) {
	if (g.sizes[1] + 2 * BS <= 64)
		launch_step2d_t<BS, 64>(cur, nxt, g, tabs, iso, st, kname, faces);
	else
		launch_step2d_t<BS, 256>(cur, nxt, g, tabs, iso, st, kname, faces);
}

bool step2d_supported(const Geo& g) {
	return g.D == 2 && g.M == 5 && g.bs >= 1 && g.bs <= kStep2dMaxBs && g.sizes[0] >= 1 && g.sizes[1] >= 1;
}

bool step2d_iso_supported(const Geo& g) {
	return step2d_supported(g) && g.bs <= 3 && g.cs * 8 < (1LL << 32);
}

bool launch_step2d(const double* cur, double* nxt, const Geo& g, const AxisTable* tabs, const IsoAxis* iso,
                   hipStream_t st, const char** kname, const Face2* faces) {
	if (!step2d_supported(g)) return false;
	if (iso && !step2d_iso_supported(g)) iso = nullptr;
	if (faces && faces->on && (!iso || g.sizes[1] < g.bs + 1)) return false;  // y faces: isotropic kernel only
	switch (g.bs) {
	case 1: launch_step2d_bs<1>(cur, nxt, g, tabs, iso, st, kname, faces); return true;
	case 2: launch_step2d_bs<2>(cur, nxt, g, tabs, iso, st, kname, faces); return true;
	case 3: launch_step2d_bs<3>(cur, nxt, g, tabs, iso, st, kname, faces); return true;
	case 4: launch_step2d_bs<4>(cur, nxt, g, tabs, iso, st, kname, faces); return true;
	case 5: launch_step2d_bs<5>(cur, nxt, g, tabs, iso, st, kname, faces); return true;
	default: return false;
	}
}

}  // namespace gcmx
