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
