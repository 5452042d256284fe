// kernels_xyz.hip -- the one-pass 3-D time step (X, Y and Z stages of
// cubic::Engine::nextTimeStep, Engine.cpp:90-121, fused into one kernel).
// Arithmetic identical to k_stage_generic / the reference stage
// (engine/cubic/GridCharacteristicMethod.hpp:42-52) through node_update (iso.hpp).
#include "iso.hpp"

#include <cstring>
#include <type_traits>

namespace gcmx {

// ------------------------------------------------------------- fused xyz --

// The whole time step in ONE pass (X stage, then Y, then Z, as
// Engine::nextTimeStep orders them, Engine.cpp:90-121): block = one x plane, a
// chunk of y rows and the whole z row.  Each thread marches y; at row y it
//   * computes the X stage of row y+BS straight from the input layer (its
//     2*BS+1 x-neighbours are plain loads; the neighbouring planes' blocks read
//     the same lines, so they come from L2 / Infinity Cache, not HBM),
//   * pushes that X result into a register window of 2*BS+1 rows and runs the
//     Y stage of row y,
//   * hands the Y result to the Z stage through double-buffered LDS.
// HBM traffic: the input layer once, the output layer once (144 B/node/step).
// Reads `in` (all components, x ghost planes valid), writes `outl`.
//
// Schedule (measured A/B on MI355X): the loop is rotated (Y, Z,
// stores, then the X stage of the row that enters the window); the X stage
// loads one characteristic pair (10 values) at a time with the next pair in
// flight, which keeps the kernel at 128 VGPRs (two 512-thread blocks per CU);
// the first pair of the next row is issued before this row's stores, so its
// vmcnt wait never includes the stores (loads and stores retire in order on
// gfx950); the output is written with non-temporal stores.
// Precondition: every y/z ghost of both layers is zero, so the intermediate
// results at ghost rows / columns are the constant 0.0.
#ifndef GCMX_XYZ_MINWAVES  // tuning builds only (scripts/ab_build.sh)
#define GCMX_XYZ_MINWAVES 4
#endif
#ifndef GCMX_XYZ_CHUNK
#define GCMX_XYZ_CHUNK 128
#endif
#ifndef GCMX_XYZ_UNROLL
#define GCMX_XYZ_UNROLL 1
#endif
#ifndef GCMX_XYZ_PIPE  // 1: k_step_pipe for borderSize <= 2 and floor(q) == 0
#define GCMX_XYZ_PIPE 0
#endif
#ifndef GCMX_XYZ_TX2  // 1: k_step_tx2 (two x planes per thread) for borderSize <= 2
#define GCMX_XYZ_TX2 1
#endif

// UNI: the launch has Z == ZT (no idle lanes) and the three axes' tables are
// identical (isotropic medium, equal h): one IsoAxis in scalar registers for all
// three stages and no idle-lane selects.
template <int BS, int ZT, bool KF0, bool UNI>
__global__ __launch_bounds__(ZT, GCMX_XYZ_MINWAVES) void k_fused_xyz(
    const double* __restrict__ in, double* __restrict__ outl, Geo g, IsoAxis AX, IsoAxis AY_,
    IsoAxis AZ_, int x0, int chunk, int nplanes) {
	const IsoAxis& AY = UNI ? AX : AY_;
	const IsoAxis& AZ = UNI ? AX : AZ_;
	constexpr unsigned WMX = iso_window(0);
	constexpr unsigned CMX = iso_center_only(0);
	constexpr unsigned WMY = iso_window(1);
	constexpr unsigned CMY = iso_center_only(1);
	constexpr int NWY = popc9(WMY);
	constexpr int NCY = popc9(CMY);
	constexpr unsigned WMZ = iso_window(2);
	constexpr int NWZ = popc9(WMZ);
	constexpr int W = 2 * BS + 1;
	constexpr int LW = ZT + 2 * BS;
	__shared__ double lds[2][NWZ][LW];

	const int z = threadIdx.x;
	const int Y = g.sizes[1], Z = g.sizes[2];
	// 1-D grid of nchunks * nplanes blocks.  Blocks are dealt round-robin over
	// the 8 XCDs (b % 8 share one, MI355X_MICROARCH.md §Workgroup dispatch): give
	// each XCD a contiguous run of (chunk, plane) pairs in chunk-major order, so
	// the 2*BS+1 x-neighbour planes a block re-reads were loaded by blocks of the
	// same XCD, i.e. hit its L2.  Placement only; any mapping is correct.
	int x, yb;
	{
		const int nx = (int)nplanes, T = (int)gridDim.x, b = (int)blockIdx.x;
		const int p = (T % 8 == 0) ? (b % 8) * (T / 8) + b / 8 : b;
		x = x0 + p % nx;
		yb = (p / nx) * chunk;
	}
	const int ye = min(yb + chunk, Y);
	const bool live = UNI || z < Z;
	const int zc = live ? z : Z - 1;  // idle lanes shadow a valid column
	const unsigned stx = (unsigned)g.stride[0];
	const unsigned sty = (unsigned)g.stride[1];
	const unsigned plane = (unsigned)(g.origin + x * g.stride[0]);
	const unsigned base = plane + zc;
	const Planes src(in, g.cs);
	const PlanesW out_p(outl, g.cs);

	if (z < 2 * BS) {  // ghost slots of both LDS row buffers: zero, never overwritten
		const int gslot = (z < BS) ? z : (Z + z);
#pragma unroll
		for (int q = 0; q < NWZ; q++) {
			lds[0][q][gslot] = 0.0;
			lds[1][q][gslot] = 0.0;
		}
	}

	// X stage of row r, loaded one characteristic pair (10 values) at a time with
	// the next pair in flight: at most two pairs are live in registers.
	typedef double PairWin[2][W];
	auto pair_load = [&](auto PC, PairWin& w, unsigned o) {
		constexpr int P = decltype(PC)::value;
#pragma unroll
		for (int k = 0; k < W; k++) {
			w[0][k] = src.ld(pair_vel(0, P), o + (unsigned)(k - BS) * stx);
			w[1][k] = src.ld(pair_sig(0, P), o + (unsigned)(k - BS) * stx);
		}
	};
	auto pair_acc = [&](auto PC, const PairWin& w) {
		constexpr int P = decltype(PC)::value;
		return [&w](int j, int o) { return j == pair_vel(0, P) ? w[0][BS + o] : w[1][BS + o]; };
	};
	auto sched_fence = [] { __builtin_amdgcn_sched_barrier(0); };
	using P0 = std::integral_constant<int, 0>;
	using P1 = std::integral_constant<int, 1>;
	using P2 = std::integral_constant<int, 2>;
	// wa holds pair 0 of row r (already issued); loads pairs 1, 2 and the
	// node-only components as it goes.
	auto x_stage_rest = [&](PairWin& wa, int r, double (&xr)[9]) {
		const unsigned o = base + (unsigned)r * sty;
		PairWin wb;
		pair_load(P1{}, wb, o);
		double rr[9], n0[9], cv[9];
		pair_update<0, BS, KF0, 0>(AX, pair_acc(P0{}, wa), rr[0], rr[1]);
		n0[pair_vel(0, 0)] = wa[0][BS];
		n0[pair_sig(0, 0)] = wa[1][BS];
		sched_fence();
		pair_load(P2{}, wa, o);
		pair_update<0, BS, KF0, 1>(AX, pair_acc(P1{}, wb), rr[2], rr[3]);
		n0[pair_vel(0, 1)] = wb[0][BS];
		n0[pair_sig(0, 1)] = wb[1][BS];
		sched_fence();
#pragma unroll
		for (int j = 0; j < 9; j++)
			if ((CMX >> j) & 1u) cv[j] = src.ld(j, o);
		pair_update<0, BS, KF0, 2>(AX, pair_acc(P2{}, wa), rr[4], rr[5]);
		n0[pair_vel(0, 2)] = wa[0][BS];
		n0[pair_sig(0, 2)] = wa[1][BS];
		sched_fence();
		center_update<0>(AX, [&](int j) { return ((WMX >> j) & 1u) ? n0[j] : cv[j]; }, rr);
		u1_apply<0>(AX, rr, xr);
	};
	auto x_load_a = [&](PairWin& wa, int r) { pair_load(P0{}, wa, base + (unsigned)r * sty); };

	// Y window over X results of rows y-BS..y+BS; node-only components of rows
	// y..y+BS wait in a small delay line.
	double win[NWY][W];
	double cen[BS + 1][NCY > 0 ? NCY : 1];
	auto push = [&](const double (&xr)[9], int slot) {  // slot: window index of the row
#pragma unroll
		for (int j = 0; j < 9; j++) {
			if ((WMY >> j) & 1u) win[wslot(WMY, j)][slot] = xr[j];
			if ((CMY >> j) & 1u) {
				if (slot >= BS) cen[slot - BS][wslot(CMY, j)] = xr[j];
			}
		}
	};
	// Rotated schedule: the loads of an X row are issued at the END of an
	// iteration and consumed after the next iteration's stores, so in every path
	// into the loop they are older than 9 stores and the compiler's vmcnt waits
	// never include the stores' completion.  Stores, LDS writes and the Z stage
	// are unconditional (idle lanes z >= Z write 0.0 into the first z ghost, which
	// the precondition keeps zero), and the in-loop X rows are loaded without a
	// branch: rows outside [0, Y) are zero ghost rows, clamped into the plane.
	// prologue: X results of rows yb-BS .. yb+BS
#pragma unroll
	for (int k = 0; k < W; k++) {
		const int r = yb - BS + k;
		double xr[9];
		if (r >= 0 && r < Y) {
			PairWin wa;
			x_load_a(wa, r);
			x_stage_rest(wa, r, xr);
		} else {
#pragma unroll
			for (int j = 0; j < 9; j++) xr[j] = 0.0;
		}
		push(xr, k);
	}
	auto clamp_row = [&](int r) { return r < Y + BS - 1 ? r : Y + BS - 1; };
	const unsigned zo = live ? (unsigned)z : (unsigned)Z;

	int buf = 0;
#pragma unroll GCMX_XYZ_UNROLL
	for (int y = yb; y < ye; y++) {
		double yv[9];
		node_update<1, BS, KF0>(
		    AY, [&](int j, int o) { return win[wslot(WMY, j)][BS + o]; },
		    [&](int j) { return ((WMY >> j) & 1u) ? win[wslot(WMY, j)][BS] : cen[0][wslot(CMY, j)]; },
		    yv);
#pragma unroll
		for (int j = 0; j < 9; j++)
			if ((WMZ >> j) & 1u) lds[buf][wslot(WMZ, j)][BS + z] = live ? yv[j] : 0.0;
		PairWin wa_next;
		__syncthreads();
		{
			double zv[9];
			node_update<2, BS, KF0>(
			    AZ, [&](int j, int o) { return lds[buf][wslot(WMZ, j)][BS + z + o]; },
			    [&](int j) { return ((WMZ >> j) & 1u) ? lds[buf][wslot(WMZ, j)][BS + z] : yv[j]; }, zv);
			const unsigned offo = plane + (unsigned)y * sty + zo;
			// next row's first pair: loads older than this row's stores
			sched_fence();
			x_load_a(wa_next, clamp_row(y + BS + 1));
			sched_fence();
#pragma unroll
			for (int c = 0; c < 9; c++) out_p.st_nt(c, offo, live ? zv[c] : 0.0);
		}
		buf ^= 1;
#pragma unroll
		for (int q = 0; q < NWY; q++)
#pragma unroll
			for (int o = 0; o < W - 1; o++) win[q][o] = win[q][o + 1];
#pragma unroll
		for (int k = 0; k < BS; k++)
#pragma unroll
			for (int q = 0; q < (NCY > 0 ? NCY : 1); q++) cen[k][q] = cen[k + 1][q];
		{  // X stage of row y+BS+1 (zero ghost rows give zero) -> window slot W-1
			double xr[9];
			sched_fence();
			x_stage_rest(wa_next, clamp_row(y + BS + 1), xr);
			push(xr, W - 1);
			sched_fence();
		}
	}
}

// ------------------------------------------------------- pipelined step --

// Component j of the axis-S stage belongs to characteristic pair pair_of(S, j)
// (as its velocity or its stress component); -1 for node-only components.
__host__ __device__ constexpr int pair_of(int S, int j) {
	return (j == pair_vel(S, 0) || j == pair_sig(S, 0)) ? 0
	     : (j == pair_vel(S, 1) || j == pair_sig(S, 1)) ? 1
	     : (j == pair_vel(S, 2) || j == pair_sig(S, 2)) ? 2 : -1;
}

// One component along the marching (y) line with the Newton differences SHARED
// between neighbouring nodes.  With forward differences on the line
//   D0_k = S_k,  Di_k = (D(i-1)_{k+1} - D(i-1)_k) * c_{i-1}
// the foot on the +y side of node y interpolates (minMaxInterpolate,
// EqualDistanceLineInterpolator.hpp:56-71, floor(q) == 0)
//   ((S_y + D1_y) + D2_y) ...            -- the reference's own operations, and
// the foot on the -y side (values S_y, S_{y-1}, S_{y-2}, ...) has
//   d_i = (-1)^i Di_{y-i}, so ((S_y - D1_{y-1}) + D2_{y-2}) ...
// because a - b == -(b - a) and (-x) * c == -(x * c) in IEEE arithmetic (up to
// the sign of an exact zero, which IEEE equality ignores -- DESIGN.md §3.2).
// Every difference is computed once, when the row that completes it enters,
// instead of once per foot: 2 * BS subtract/multiply per component and node
// instead of 4 * BS.  The limiter bounds of the -y foot, min/max(S_y, S_{y-1}),
// are the +y bounds of row y-1.
template <int BS>
struct YLine {
	double s[BS];        // S_y .. S_{y+BS-1}
	double d[BS][BS];    // d[i-1][k] = Di_{y-i+k}, k = 0..BS-1
	double mxm, mnm;     // bounds of the -y foot of row y: max/min(S_y, S_{y-1})
	double sn, nd[BS];   // the entering row S_{y+BS} and the differences it completes
	__device__ __forceinline__ void clear() {
#pragma unroll
		for (int k = 0; k < BS; k++) s[k] = 0.0;
#pragma unroll
		for (int i = 0; i < BS; i++)
#pragma unroll
			for (int k = 0; k < BS; k++) d[i][k] = 0.0;
		mxm = mnm = 0.0;
	}
	// S_{y+BS} enters: D1_{y+BS-1}, D2_{y+BS-2}, ..., D(BS)_y.
	__device__ __forceinline__ void enter(double v, const double* c) {
		sn = v;
		nd[0] = (v - s[BS - 1]) * c[0];
#pragma unroll
		for (int i = 1; i < BS; i++) nd[i] = (nd[i - 1] - d[i - 1][BS - 1]) * c[i];
	}
	// The two interpolants of row y (minus: foot on the -y side, U rows 2P).
	__device__ __forceinline__ void feet(double& im, double& ip, double& mxp, double& mnp) const {
		const double s1 = (BS >= 2) ? s[BS >= 2 ? 1 : 0] : sn;  // S_{y+1}
		double a = s[0];
#pragma unroll
		for (int i = 0; i < BS; i++) a += (i + 1 < BS) ? d[i][(i + 1) < BS ? i + 1 : 0] : nd[BS - 1];
		double b = s[0];
#pragma unroll
		for (int i = 0; i < BS; i++) b = (i % 2 == 0) ? b - d[i][0] : b + d[i][0];
		mxp = vmax(s[0], s1);
		mnp = vmin(s[0], s1);
		ip = vmin(vmax(a, mnp), mxp);
		im = vmin(vmax(b, mnm), mxm);
	}
	__device__ __forceinline__ void shift(double mxp, double mnp) {
#pragma unroll
		for (int k = 0; k + 1 < BS; k++) s[k] = s[k + 1];
		s[BS - 1] = sn;
#pragma unroll
		for (int i = 0; i < BS; i++) {
#pragma unroll
			for (int k = 0; k + 1 < BS; k++) d[i][k] = d[i][k + 1];
			d[i][BS - 1] = nd[i];
		}
		mxm = mxp;
		mnm = mnp;
	}
};

#ifndef GCMX_PIPE_MINWAVES  // waves per SIMD the register budget is sized for
#define GCMX_PIPE_MINWAVES 2
#endif
#ifndef GCMX_PIPE_UNROLL
#define GCMX_PIPE_UNROLL 1
#endif

// The whole time step in one pass, software-pipelined (the default 3-D step for
// borderSize 1-2 and Courant numbers < 1, i.e. floor(q) == 0 on every axis).
// Same block/plane/row decomposition and arithmetic as k_fused_xyz, but
//   * the X-stage inputs of the NEXT row (all 6*(2*BS+1) + 3 values) are loaded
//     one whole iteration ahead, so the Y and Z stages of this row (and the other
//     waves' work) hide their latency; the register budget of 2 waves/SIMD
//     (256 VGPRs) holds that row, the Y-line state and the temporaries;
//   * the Y stage shares its Newton differences along y (YLine).
// Reads `in` (all components, x ghost planes valid), writes `outl`.
// Precondition as k_fused_xyz: y/z ghosts of both layers are zero.
template <int BS, int ZT, bool UNI>
__global__ __launch_bounds__(ZT, GCMX_PIPE_MINWAVES) void k_step_pipe(
    const double* __restrict__ in, double* __restrict__ outl, Geo g, IsoAxis AX, IsoAxis AY_,
    IsoAxis AZ_, int x0, int chunk, int nplanes) {
	const IsoAxis& AY = UNI ? AX : AY_;
	const IsoAxis& AZ = UNI ? AX : AZ_;
	constexpr unsigned WMX = iso_window(0);
	constexpr unsigned CMX = iso_center_only(0);
	constexpr int NCX = popc9(CMX);
	constexpr unsigned WMY = iso_window(1);
	constexpr unsigned CMY = iso_center_only(1);
	constexpr int NWY = popc9(WMY);
	constexpr int NCY = popc9(CMY);
	constexpr unsigned WMZ = iso_window(2);
	constexpr int NWZ = popc9(WMZ);
	constexpr int W = 2 * BS + 1;
	constexpr int LW = ZT + 2 * BS;
	static_assert(NWY == 6 && NCX >= 1 && NCY >= 1, "isotropic structure");
	__shared__ double lds[2][NWZ][LW];

	const int z = threadIdx.x;
	const int Y = g.sizes[1], Z = g.sizes[2];
	int x, yb;
	{  // XCD-aware chunk-major block order (see k_fused_xyz)
		const int nx = (int)nplanes, T = (int)gridDim.x, b = (int)blockIdx.x;
		const int p = (T % 8 == 0) ? (b % 8) * (T / 8) + b / 8 : b;
		x = x0 + p % nx;
		yb = (p / nx) * chunk;
	}
	const int ye = min(yb + chunk, Y);
	const bool live = UNI || z < Z;
	const int zc = live ? z : Z - 1;
	const unsigned stx = (unsigned)g.stride[0];
	const unsigned sty = (unsigned)g.stride[1];
	const unsigned plane = (unsigned)(g.origin + x * g.stride[0]);
	const unsigned base = plane + zc;
	const Planes src(in, g.cs);
	const PlanesW out_p(outl, g.cs);

	if (z < 2 * BS) {
		const int gslot = (z < BS) ? z : (Z + z);
#pragma unroll
		for (int q = 0; q < NWZ; q++) {
			lds[0][q][gslot] = 0.0;
			lds[1][q][gslot] = 0.0;
		}
	}

	// X-stage inputs of one row.
	struct XIn {
		double w[3][2][W];  // pair P: velocity / stress component at x-offsets -BS..BS
		double c[NCX];      // node-only components at the node
	};
	auto x_load = [&](XIn& v, int r) {
		const unsigned o = base + (unsigned)r * sty;
#pragma unroll
		for (int P = 0; P < 3; P++)
#pragma unroll
			for (int k = 0; k < W; k++) {
				v.w[P][0][k] = src.ld(pair_vel(0, P), o + (unsigned)(k - BS) * stx);
				v.w[P][1][k] = src.ld(pair_sig(0, P), o + (unsigned)(k - BS) * stx);
			}
#pragma unroll
		for (int j = 0; j < 9; j++)
			if ((CMX >> j) & 1u) v.c[wslot(CMX, j)] = src.ld(j, o);
	};
	auto x_stage = [&](const XIn& v, double (&xr)[9]) {
		double rr[9];
		auto wv = [&](int j, int o) {
			const int P = pair_of(0, j);
			return j == pair_vel(0, P) ? v.w[P][0][BS + o] : v.w[P][1][BS + o];
		};
		pair_update<0, BS, true, 0>(AX, wv, rr[0], rr[1]);
		pair_update<0, BS, true, 1>(AX, wv, rr[2], rr[3]);
		pair_update<0, BS, true, 2>(AX, wv, rr[4], rr[5]);
		center_update<0>(AX, [&](int j) { return ((WMX >> j) & 1u) ? wv(j, 0) : v.c[wslot(CMX, j)]; }, rr);
		u1_apply<0>(AX, rr, xr);
	};
	auto sched_fence = [] { __builtin_amdgcn_sched_barrier(0); };

	YLine<BS> yl[NWY];
	double cen[BS + 1][NCY];  // node-only Y components of rows y .. y+BS
#pragma unroll
	for (int q = 0; q < NWY; q++) yl[q].clear();
#pragma unroll
	for (int k = 0; k <= BS; k++)
#pragma unroll
		for (int q = 0; q < NCY; q++) cen[k][q] = 0.0;
	auto ycoef = [&](int j) { return pair_of(1, j) == 0 ? AY.c1 : AY.c2; };
	// Row y + BS enters the y line (its X result xr).
	auto enter = [&](const double (&xr)[9]) {
#pragma unroll
		for (int j = 0; j < 9; j++) {
			if ((WMY >> j) & 1u) yl[wslot(WMY, j)].enter(xr[j], ycoef(j));
			if ((CMY >> j) & 1u) cen[BS][wslot(CMY, j)] = xr[j];
		}
	};
	double mxp[NWY], mnp[NWY];
	auto advance = [&]() {
#pragma unroll
		for (int q = 0; q < NWY; q++) yl[q].shift(mxp[q], mnp[q]);
#pragma unroll
		for (int k = 0; k < BS; k++)
#pragma unroll
			for (int q = 0; q < NCY; q++) cen[k][q] = cen[k + 1][q];
	};
	auto clamp_row = [&](int r) { return r < Y + BS - 1 ? r : Y + BS - 1; };

	// prologue: rows yb-BS .. yb+BS-1 enter the line (rows < 0 are zero ghosts)
	for (int k = 0; k < 2 * BS; k++) {
		const int r = yb - BS + k;
		double xr[9];
		if (r >= 0) {
			XIn v;
			x_load(v, clamp_row(r));
			x_stage(v, xr);
		} else {
#pragma unroll
			for (int j = 0; j < 9; j++) xr[j] = 0.0;
		}
		enter(xr);
#pragma unroll
		for (int q = 0; q < NWY; q++) {  // +y bounds of row r - BS + 1 ... only the last matters
			const double s1 = (BS >= 2) ? yl[q].s[BS >= 2 ? 1 : 0] : yl[q].sn;
			mxp[q] = vmax(yl[q].s[0], s1);
			mnp[q] = vmin(yl[q].s[0], s1);
		}
		advance();
	}
	XIn pf;
	x_load(pf, clamp_row(yb + BS));
	const unsigned zo = live ? (unsigned)z : (unsigned)Z;

	int buf = 0;
	auto row = [&](int y) {
		double xr[9];
		sched_fence();
		x_stage(pf, xr);  // row y + BS
		sched_fence();
		x_load(pf, clamp_row(y + BS + 1));  // consumed by the next iteration
		sched_fence();
		enter(xr);
		double yv[9];
		{
			double im[NWY], ip[NWY];
#pragma unroll
			for (int q = 0; q < NWY; q++) yl[q].feet(im[q], ip[q], mxp[q], mnp[q]);
			double r[9];
			auto IM = [&](int j) { return im[wslot(WMY, j)]; };
			auto IP = [&](int j) { return ip[wslot(WMY, j)]; };
			r[0] = RowSum<1, false, 0>::go(AY, IM, 0.0, true);
			r[1] = RowSum<1, false, 1>::go(AY, IP, 0.0, true);
			r[2] = RowSum<1, false, 2>::go(AY, IM, 0.0, true);
			r[3] = RowSum<1, false, 3>::go(AY, IP, 0.0, true);
			r[4] = RowSum<1, false, 4>::go(AY, IM, 0.0, true);
			r[5] = RowSum<1, false, 5>::go(AY, IP, 0.0, true);
			center_update<1>(
			    AY, [&](int j) { return ((WMY >> j) & 1u) ? yl[wslot(WMY, j)].s[0] : cen[0][wslot(CMY, j)]; }, r);
			u1_apply<1>(AY, r, yv);
		}
#pragma unroll
		for (int j = 0; j < 9; j++)
			if ((WMZ >> j) & 1u) lds[buf][wslot(WMZ, j)][BS + z] = live ? yv[j] : 0.0;
		__syncthreads();
		{
			double zv[9];
			node_update<2, BS, true>(
			    AZ, [&](int j, int o) { return lds[buf][wslot(WMZ, j)][BS + z + o]; },
			    [&](int j) { return ((WMZ >> j) & 1u) ? lds[buf][wslot(WMZ, j)][BS + z] : yv[j]; }, zv);
			const unsigned offo = plane + (unsigned)y * sty + zo;
#pragma unroll
			for (int c = 0; c < 9; c++) out_p.st_nt(c, offo, live ? zv[c] : 0.0);
		}
		buf ^= 1;
		advance();
	};
	// Unrolled by hand (a loop holding a barrier is not unrolled with a
	// remainder by the compiler): the shifts of the y-line state become
	// register renames inside the unrolled body.
	int y = yb;
	for (; y + GCMX_PIPE_UNROLL <= ye; y += GCMX_PIPE_UNROLL) {
#pragma unroll
		for (int u = 0; u < GCMX_PIPE_UNROLL; u++) row(y + u);
	}
	for (; y < ye; y++) row(y);
}

// ------------------------------------------------ two planes per thread --

#ifndef GCMX_TX2_MINWAVES
#define GCMX_TX2_MINWAVES 2
#endif
#ifndef GCMX_TX2_XSHARE  // share the X-stage Newton differences of the two nodes
#define GCMX_TX2_XSHARE 1
#endif
#ifndef GCMX_TX2_PINGPONG  // opposite segment orders on the two waves of a SIMD
#define GCMX_TX2_PINGPONG 0
#endif
#ifndef GCMX_TX2_AHEAD  // load pairs issued one segment ahead of the X stage (1 or 2)
#define GCMX_TX2_AHEAD 2
#endif
#ifndef GCMX_TX2_DIAG  // tuning builds only: per-wave phase cycle counters (s_memtime)
#define GCMX_TX2_DIAG 0
#endif
#if GCMX_TX2_DIAG
__device__ unsigned long long g_tx2_diag[16][8];  // [wave in block][phase]: cycles summed over blocks
#define TX2_T(i)                                                   \
	do {                                                           \
		const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
		dt_[i] += now_ - tprev_;                                   \
		tprev_ = now_;                                             \
	} while (0)
#else
#define TX2_T(i) \
	do {         \
	} while (0)
#endif

// The whole time step in one pass with TWO adjacent x planes per thread
// (x, x+1 at one z).  The X stages of both nodes read the 2*BS+2 planes
// x-BS .. x+1+BS: 6*(2*BS+2) + 2*3 loads per two nodes instead of
// 2*(6*(2*BS+1) + 3) -- the x-neighbour re-reads are L2->CU bandwidth, which
// bounds the one-plane kernel (tools/xyz_probe.hip: 33 loads + 9 stores per node
// take 1.2-1.3x the time of the compulsory 9 + 9).  Arithmetic per node is
// k_fused_xyz's (node_update / pair_update).  Registers hold the two Y windows;
// the node-only Y components of rows y..y+BS (read back by the same thread
// only) live in an LDS ring, and the Z exchange is one LDS buffer per node
// with two barriers per row.  One 512-thread block per CU (2 waves/SIMD).
// If the launch has an odd number of planes the last thread's second node is
// computed from clamped (valid) planes and not stored.
template <int BS, int ZT, bool KF0, bool UNI>
__global__ __launch_bounds__(ZT, GCMX_TX2_MINWAVES) void k_step_tx2(
    const double* __restrict__ in, double* __restrict__ outl, Geo g, IsoAxis AX, IsoAxis AY_,
    IsoAxis AZ_, int x0, int chunk, int nplanes) {
	const IsoAxis& AY = UNI ? AX : AY_;
	const IsoAxis& AZ = UNI ? AX : AZ_;
	constexpr unsigned WMX = iso_window(0);
	constexpr unsigned CMX = iso_center_only(0);
	constexpr int NCX = popc9(CMX);
	constexpr unsigned WMY = iso_window(1);
	constexpr unsigned CMY = iso_center_only(1);
	constexpr int NWY = popc9(WMY);
	constexpr int NCY = popc9(CMY);
	constexpr unsigned WMZ = iso_window(2);
	constexpr int NWZ = popc9(WMZ);
	constexpr int W = 2 * BS + 1;
	constexpr int WX = W + 1;  // planes x-BS .. x+1+BS
	constexpr int LW = ZT + 2 * BS;
	static_assert(NCX >= 1 && NCY >= 1, "isotropic structure");
	__shared__ double zl[2][NWZ][LW];           // Y results of both nodes (Z stage input)
	__shared__ double cl[BS + 1][2][NCY][ZT];   // node-only Y components, rows y..y+BS (ring)

	const int z = threadIdx.x;
	const int Y = g.sizes[1], Z = g.sizes[2];
	int x, yb;
	{  // XCD-aware chunk-major block order (see k_fused_xyz) over plane pairs
		const int npair = (nplanes + 1) / 2, T = (int)gridDim.x, b = (int)blockIdx.x;
		const int p = (T % 8 == 0) ? (b % 8) * (T / 8) + b / 8 : b;
		x = x0 + 2 * (p % npair);
		yb = (p / npair) * chunk;
	}
	const bool two = x + 1 < x0 + nplanes;
	const int ye = min(yb + chunk, Y);
	const bool live = UNI || z < Z;
	const int zc = live ? z : Z - 1;
	const unsigned stx = (unsigned)g.stride[0];
	const unsigned sty = (unsigned)g.stride[1];
	const unsigned plane = (unsigned)(g.origin + x * g.stride[0]);
	const unsigned base = plane + zc;
	const Planes src(in, g.cs);
	const PlanesW out_p(outl, g.cs);
	// element offset of plane x - BS + k (the last one clamped when x + 1 is not ours)
	auto xoff = [&](int k) {
		const int d = (k == WX - 1 && !two) ? BS : k - BS;
		return (unsigned)d * stx;
	};

	if (z < 2 * BS) {
		const int gslot = (z < BS) ? z : (Z + z);
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int q = 0; q < NWZ; q++) zl[t][q][gslot] = 0.0;
	}

	typedef double PairWin[2][WX];  // [vel/sig][plane]
	auto pair_load = [&](auto PC, PairWin& w, unsigned o) {
		constexpr int P = decltype(PC)::value;
#pragma unroll
		for (int k = 0; k < WX; k++) {
			w[0][k] = src.ld(pair_vel(0, P), o + xoff(k));
			w[1][k] = src.ld(pair_sig(0, P), o + xoff(k));
		}
	};
	auto pair_acc = [&](auto PC, const PairWin& w, int t) {
		constexpr int P = decltype(PC)::value;
		return [&w, t](int j, int o) { return j == pair_vel(0, P) ? w[0][t + BS + o] : w[1][t + BS + o]; };
	};
	// Rows 2P, 2P+1 of both nodes.  With floor(q) == 0 the Newton differences
	// along x are shared between the two nodes (YLine's identity: the -x foot
	// uses (-1)^i Di_{m-i}); otherwise per node through pair_update.
	auto pair_rows = [&](auto PC, const PairWin& w, double (&rr)[2][9]) {
		constexpr int P = decltype(PC)::value;
		if constexpr (KF0 && GCMX_TX2_XSHARE) {
			const double* c = (P == 0) ? AX.c1 : AX.c2;
			double im[2][2], ip[2][2];  // [vel/sig][node]
#pragma unroll
			for (int v = 0; v < 2; v++) {
				double D[BS + 1][WX];
#pragma unroll
				for (int k = 0; k < WX; k++) D[0][k] = w[v][k];
#pragma unroll
				for (int i = 1; i <= BS; i++)
#pragma unroll
					for (int k = 0; k + i < WX; k++) D[i][k] = (D[i - 1][k + 1] - D[i - 1][k]) * c[i - 1];
				double mx[WX - 1], mn[WX - 1];  // bounds of segment (k, k+1), node value first
#pragma unroll
				for (int t = 0; t < 2; t++) {
					const int m = t + BS;
					double a = D[0][m], b = D[0][m];
#pragma unroll
					for (int i = 1; i <= BS; i++) {
						a += D[i][m];
						b = (i % 2) ? b - D[i][m - i] : b + D[i][m - i];
					}
					const double mxp = vmax(D[0][m], D[0][m + 1]), mnp = vmin(D[0][m], D[0][m + 1]);
					double mxm, mnm;
					if (t == 1) {  // the -x segment of node 1 is the +x segment of node 0
						mxm = mx[m - 1];
						mnm = mn[m - 1];
					} else {
						mxm = vmax(D[0][m], D[0][m - 1]);
						mnm = vmin(D[0][m], D[0][m - 1]);
					}
					mx[m] = mxp;
					mn[m] = mnp;
					ip[v][t] = vmin(vmax(a, mnp), mxp);
					im[v][t] = vmin(vmax(b, mnm), mxm);
				}
			}
#pragma unroll
			for (int t = 0; t < 2; t++) {
				rr[t][2 * P] = RowSum<0, false, 2 * P>::go(
				    AX, [&](int j) { return j == pair_vel(0, P) ? im[0][t] : im[1][t]; }, 0.0, true);
				rr[t][2 * P + 1] = RowSum<0, false, 2 * P + 1>::go(
				    AX, [&](int j) { return j == pair_vel(0, P) ? ip[0][t] : ip[1][t]; }, 0.0, true);
			}
		} else {
#pragma unroll
			for (int t = 0; t < 2; t++)
				pair_update<0, BS, KF0, P>(AX, pair_acc(PC, w, t), rr[t][2 * P], rr[t][2 * P + 1]);
		}
	};
	auto sched_fence = [] { __builtin_amdgcn_sched_barrier(0); };
	using P0 = std::integral_constant<int, 0>;
	using P1 = std::integral_constant<int, 1>;
	using P2 = std::integral_constant<int, 2>;
	// X stage of row r for both nodes; wa holds pair 0 (already issued).
	// The X-stage inputs of a row issued ahead of its X stage: pair 0 (AHEAD 1)
	// or pairs 0 and 1 (AHEAD 2); the rest is issued when the X stage starts.
	struct XPre {
		PairWin a;
		PairWin b[GCMX_TX2_AHEAD >= 2 ? 1 : 1];
	};
	auto x_stage_rest = [&](XPre& pre, int r, double (&xr)[2][9]) {
		const unsigned o = base + (unsigned)r * sty;
		PairWin& wa = pre.a;
		PairWin& wb = pre.b[0];
		double rr[2][9], n0[2][9], cv[2][9];
		PairWin wc;
		if constexpr (GCMX_TX2_AHEAD >= 2) {  // pair 2 and the node-only components now
			pair_load(P2{}, wc, o);
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++)
					if ((CMX >> j) & 1u) cv[t][j] = src.ld(j, o + (unsigned)t * stx);
			sched_fence();
		} else {
			pair_load(P1{}, wb, o);
		}
		pair_rows(P0{}, wa, rr);
#pragma unroll
		for (int t = 0; t < 2; t++) {
			n0[t][pair_vel(0, 0)] = wa[0][t + BS];
			n0[t][pair_sig(0, 0)] = wa[1][t + BS];
		}
		sched_fence();
		if constexpr (GCMX_TX2_AHEAD < 2) pair_load(P2{}, wc, o);
		pair_rows(P1{}, wb, rr);
#pragma unroll
		for (int t = 0; t < 2; t++) {
			n0[t][pair_vel(0, 1)] = wb[0][t + BS];
			n0[t][pair_sig(0, 1)] = wb[1][t + BS];
		}
		sched_fence();
		if constexpr (GCMX_TX2_AHEAD < 2) {
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++)
					if ((CMX >> j) & 1u) cv[t][j] = src.ld(j, o + (unsigned)t * stx);
		}
		pair_rows(P2{}, wc, rr);
#pragma unroll
		for (int t = 0; t < 2; t++) {
			n0[t][pair_vel(0, 2)] = wc[0][t + BS];
			n0[t][pair_sig(0, 2)] = wc[1][t + BS];
		}
		sched_fence();
#pragma unroll
		for (int t = 0; t < 2; t++) {
			center_update<0>(AX, [&](int j) { return ((WMX >> j) & 1u) ? n0[t][j] : cv[t][j]; }, rr[t]);
			u1_apply<0>(AX, rr[t], xr[t]);
		}
	};
	auto x_load_a = [&](XPre& pre, int r) {
		pair_load(P0{}, pre.a, base + (unsigned)r * sty);
		if constexpr (GCMX_TX2_AHEAD >= 2) pair_load(P1{}, pre.b[0], base + (unsigned)r * sty);
	};

	double win[2][NWY][W];
	// row r's X result enters window slot `slot`; its node-only components go to the ring
	auto push = [&](const double (&xr)[2][9], int slot, int r) {
		const int ring = (r + BS) % (BS + 1);
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int j = 0; j < 9; j++) {
				if ((WMY >> j) & 1u) win[t][wslot(WMY, j)][slot] = xr[t][j];
				if ((CMY >> j) & 1u) cl[ring][t][wslot(CMY, j)][z] = xr[t][j];
			}
	};
	// prologue: X results of rows yb-BS .. yb+BS (rows < 0 or >= Y are zero ghosts)
#pragma unroll
	for (int k = 0; k < W; k++) {
		const int r = yb - BS + k;
		double xr[2][9];
		if (r >= 0 && r < Y) {
			XPre pre;
			x_load_a(pre, r);
			x_stage_rest(pre, r, xr);
		} else {
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++) xr[t][j] = 0.0;
		}
		push(xr, k, r);  // rows yb-BS, yb-BS+1 are overwritten in the ring by yb+1, yb+2
	}
	auto clamp_row = [&](int r) { return r < Y + BS - 1 ? r : Y + BS - 1; };
	const unsigned zo = live ? (unsigned)z : (unsigned)Z;

	// Ping-pong between the two waves of each SIMD (waves w and w+4 of the
	// 512-thread block share SIMD w % 4): between the barriers the first half
	// runs Z stage -> stores -> X stage of the next row, the second half X stage
	// -> Z stage -> stores, so the L2/HBM waits of one wave's X stage fall on its
	// partner's Z-stage arithmetic instead of coinciding with it.
	const bool second = __builtin_amdgcn_readfirstlane(threadIdx.x / 64) >= (ZT / 128) && GCMX_TX2_PINGPONG;
#if GCMX_TX2_DIAG
	unsigned long long dt_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
	for (int y = yb; y < ye; y++) {
		double yv[2][9];
		const int ring = (y + BS) % (BS + 1);
#pragma unroll
		for (int t = 0; t < 2; t++)
			node_update<1, BS, KF0>(
			    AY, [&](int j, int o) { return win[t][wslot(WMY, j)][BS + o]; },
			    [&](int j) { return ((WMY >> j) & 1u) ? win[t][wslot(WMY, j)][BS] : cl[ring][t][wslot(CMY, j)][z]; },
			    yv[t]);
		TX2_T(0);
		__syncthreads();  // every wave has finished reading zl (previous row's Z stage)
		TX2_T(1);
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((WMZ >> j) & 1u) zl[t][wslot(WMZ, j)][BS + z] = live ? yv[t][j] : 0.0;
		__syncthreads();
		TX2_T(2);
		XPre wa_next;
		const unsigned offo = plane + (unsigned)y * sty + zo;
		double zv[2][9];
		auto z_stage = [&]() {
#pragma unroll
			for (int t = 0; t < 2; t++)
				node_update<2, BS, KF0>(
				    AZ, [&](int j, int o) { return zl[t][wslot(WMZ, j)][BS + z + o]; },
				    [&](int j) { return ((WMZ >> j) & 1u) ? zl[t][wslot(WMZ, j)][BS + z] : yv[t][j]; }, zv[t]);
		};
		auto stores = [&]() {
#pragma unroll
			for (int c = 0; c < 9; c++) out_p.st_nt(c, offo, live ? zv[0][c] : 0.0);
			if (two) {
#pragma unroll
				for (int c = 0; c < 9; c++) out_p.st_nt(c, offo + stx, live ? zv[1][c] : 0.0);
			}
		};
		auto x_next = [&]() {  // X stage of row y+BS+1 (zero ghost rows give zero) -> window slot W-1
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int q = 0; q < NWY; q++)
#pragma unroll
					for (int o = 0; o < W - 1; o++) win[t][q][o] = win[t][q][o + 1];
			double xr[2][9];
			sched_fence();
			x_stage_rest(wa_next, clamp_row(y + BS + 1), xr);
			push(xr, W - 1, y + BS + 1);
			sched_fence();
		};
		auto load_next = [&]() {
			sched_fence();
			x_load_a(wa_next, clamp_row(y + BS + 1));
			sched_fence();
		};
		if (second) {
			load_next();
			x_next();
			TX2_T(5);
			z_stage();
			TX2_T(3);
			stores();
			TX2_T(4);
		} else {
			z_stage();
			TX2_T(3);
			load_next();  // loads older than this row's stores
			stores();
			TX2_T(4);
			x_next();
			TX2_T(5);
		}
	}
#if GCMX_TX2_DIAG
	if ((threadIdx.x & 63) == 0) {
		const int wv = threadIdx.x / 64;
		for (int i = 0; i < 8; i++) atomicAdd(&g_tx2_diag[wv][i], dt_[i]);
	}
#endif
}

// ------------------------------------------------------------- launchers --

static bool same_axis(const IsoAxis& p, const IsoAxis& q) {  // bitwise
	static_assert(sizeof(IsoAxis) == 12 * 8 + 2 * 4, "IsoAxis has padding");
	return std::memcmp(&p, &q, sizeof(IsoAxis)) == 0;
}

// Rows per block: GCMX_XYZ_CHUNK (128) while the launch still has >= 1024 blocks
// (two rounds of the 512 resident blocks, 2 per CU); thinner slabs (multi-GPU
// X slabs, the boundary planes) halve it, down to 16 rows, to keep every CU
// busy.  Each block recomputes 2*BS X rows in its prologue, so a chunk of c
// rows costs (c + 2*BS) / c of the X stage.  `req` > 0 forces a value.
static int xyz_chunk_for(int Y, int nplanes, int req) {
	int chunk = req > 0 ? req : GCMX_XYZ_CHUNK;
	if (req <= 0)
		while (chunk > 16 && (long long)((Y + chunk - 1) / chunk) * nplanes < 1024) chunk /= 2;
	return Y <= chunk ? Y : chunk;
}

template <int BS, int ZT>
static void launch_xyz_t(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                         int x1, hipStream_t st, int req_chunk) {
	const int chunk = xyz_chunk_for(g.sizes[1], x1 - x0, req_chunk);
	const int nchunks = (g.sizes[1] + chunk - 1) / chunk;
	dim3 grid(nchunks * (x1 - x0));
	bool kf0 = true;
	for (int s = 0; s < 3; s++) kf0 = kf0 && a[s].kf1 == 0 && a[s].kf2 == 0;
	const bool uni = kf0 && g.sizes[2] == ZT && same_axis(a[0], a[1]) && same_axis(a[0], a[2]);
	if constexpr (BS <= 2 && ZT <= 512) {
		if (GCMX_XYZ_TX2 && x1 - x0 >= 2) {
			const int npair = (x1 - x0 + 1) / 2;
			const int chunk2 = xyz_chunk_for(g.sizes[1], npair, req_chunk);
			dim3 grid2(((g.sizes[1] + chunk2 - 1) / chunk2) * npair);
			if (uni)
				hipLaunchKernelGGL((k_step_tx2<BS, ZT, true, true>), grid2, dim3(ZT), 0, st, in, out, g,
				                   a[0], a[1], a[2], x0, chunk2, x1 - x0);
			else if (kf0)
				hipLaunchKernelGGL((k_step_tx2<BS, ZT, true, false>), grid2, dim3(ZT), 0, st, in, out, g,
				                   a[0], a[1], a[2], x0, chunk2, x1 - x0);
			else
				hipLaunchKernelGGL((k_step_tx2<BS, ZT, false, false>), grid2, dim3(ZT), 0, st, in, out, g,
				                   a[0], a[1], a[2], x0, chunk2, x1 - x0);
			return;
		}
		if (kf0 && GCMX_XYZ_PIPE) {
			if (uni)
				hipLaunchKernelGGL((k_step_pipe<BS, ZT, true>), grid, dim3(ZT), 0, st, in, out, g, a[0],
				                   a[1], a[2], x0, chunk, x1 - x0);
			else
				hipLaunchKernelGGL((k_step_pipe<BS, ZT, false>), grid, dim3(ZT), 0, st, in, out, g, a[0],
				                   a[1], a[2], x0, chunk, x1 - x0);
			return;
		}
	}
	if (uni)
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, true, true>), grid, dim3(ZT), 0, st, in, out, g, a[0],
		                   a[1], a[2], x0, chunk, x1 - x0);
	else if (kf0)
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, true, false>), grid, dim3(ZT), 0, st, in, out, g, a[0],
		                   a[1], a[2], x0, chunk, x1 - x0);
	else
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, false, false>), grid, dim3(ZT), 0, st, in, out, g,
		                   a[0], a[1], a[2], x0, chunk, x1 - x0);
}

template <int BS>
static bool launch_xyz_bs(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                          int x1, hipStream_t st, int ch) {
	const int Z = g.sizes[2];
	if (Z <= 64) launch_xyz_t<BS, 64>(in, out, g, a, x0, x1, st, ch);
	else if (Z <= 128) launch_xyz_t<BS, 128>(in, out, g, a, x0, x1, st, ch);
	else if (Z <= 256) launch_xyz_t<BS, 256>(in, out, g, a, x0, x1, st, ch);
	else if (Z <= 512) launch_xyz_t<BS, 512>(in, out, g, a, x0, x1, st, ch);
	else launch_xyz_t<BS, 1024>(in, out, g, a, x0, x1, st, ch);
	return true;
}

#if GCMX_TX2_DIAG
extern "C" int gcmx_diag_tx2(unsigned long long* out) {  // 16 x 8 counters, then reset
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tx2_diag), sizeof(g_tx2_diag)) != hipSuccess) return -1;
	static const unsigned long long zero[16][8] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_tx2_diag), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

bool launch_fused_xyz(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                      int x1, hipStream_t st, int chunk) {
	if (!fused_supported(g) || x1 <= x0) return false;
	switch (g.bs) {
	case 1: return launch_xyz_bs<1>(in, out, g, a, x0, x1, st, chunk);
	case 2: return launch_xyz_bs<2>(in, out, g, a, x0, x1, st, chunk);
	case 3: return launch_xyz_bs<3>(in, out, g, a, x0, x1, st, chunk);
	default: return false;
	}
}

}  // namespace gcmx
