// kernels_xyz.hip -- the one-pass 3-D time step (X, Y and Z stages of
// cubic::Engine::nextTimeStep, Engine.cpp:90-121, fused into one kernel).
// Arithmetic identical to k_stage_generic / the reference stage
// (engine/cubic/GridCharacteristicMethod.hpp:42-52) through node_update (iso.hpp).
#include "iso.hpp"

#include <cstring>
#include <string>
#include <type_traits>

namespace gcmx {
// This file is compiled twice (Makefile): as the exact build (xyz_exact,
// -ffp-contract=off: the reference's separate multiply and add roundings,
// bitwise equal to the oracle) and as the FMA build (xyz_fma, -DGCMX_FMA=1
// -ffp-contract=fast: multiply-adds contracted, within the north-star fp64
// tolerance of the reference).  gcmx_set_fp_mode selects one.
#ifndef GCMX_FMA
#define GCMX_FMA 0
#endif
#if GCMX_FMA
#define GCMX_XYZ_NS xyz_fma
#define GCMX_FP_TAG ", FMA"
#else
#define GCMX_XYZ_NS xyz_exact
#define GCMX_FP_TAG ""
#endif
namespace GCMX_XYZ_NS {

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
#ifndef GCMX_XYZ_MINWAVES_BS3  // borderSize 3 (tuning builds only: 4 was the round-5 value)
#define GCMX_XYZ_MINWAVES_BS3 2
#endif
#ifndef GCMX_XYZ_TX2  // 1: k_step_tx2 (two x planes per thread) for borderSize <= 2, Z <= 512
#define GCMX_XYZ_TX2 1
#endif

// borderSize 3 runs at 2 waves per SIMD: at 4 (128 VGPRs) its windows spill 97
// VGPRs to scratch (profiles/r6/bs3_resource_usage.txt).
// UNI: the launch has Z == ZT (no idle lanes) and the three axes' tables are
// identical (isotropic medium, equal h): one IsoAxis in scalar registers for all
// three stages and no idle-lane selects.
template <int BS, int ZT, bool KF0, bool UNI>
__global__ __launch_bounds__(ZT, BS >= 3 ? GCMX_XYZ_MINWAVES_BS3 : GCMX_XYZ_MINWAVES) void k_fused_xyz(
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
		const int p = xcd_order(b, T);
		x = x0 + p % nx;
		yb = (p / nx) * chunk;
	}
	const int ye = min(yb + chunk, Y);
	const bool live = UNI || z < Z;
	const int zc = live ? z : Z - 1;  // idle lanes shadow a valid column
	const unsigned stx = (unsigned)g.stride[0];
	const unsigned sty = (unsigned)g.stride[1];
	// Plane bases in SGPRs at this block's plane x, element offsets relative to
	// them: 32-bit offsets whatever the layer's size (onepass_layout_ok)
	const long long pbase = (long long)x * g.stride[0];
	const unsigned plane = (unsigned)g.origin;  // node (x, 0, 0) from the bases
	const unsigned base = plane + zc;
	const Planes src(in + pbase, g.cs);
	const PlanesW out_p(outl + pbase, g.cs);

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

// ------------------------------------------------ two planes per thread --

#ifndef GCMX_TX2_MINWAVES
#define GCMX_TX2_MINWAVES 2
#endif
#ifndef GCMX_TX2_ZS2  // split the ahead-loads around the two nodes' Z stage + stores (-1: unless NB)
#define GCMX_TX2_ZS2 -1
#endif
#ifndef GCMX_TX2_NB  // UNI launches: Z exchange without block barriers (per-wave regions + edge ring)
#define GCMX_TX2_NB 1
#endif
#ifndef GCMX_TX2_SLEEP  // NB: s_sleep argument while a neighbour wave's edges are not there yet
#define GCMX_TX2_SLEEP 1
#endif
#ifndef GCMX_TX2_BUF  // buffer loads/stores: block-uniform offsets in SGPRs (no VALU address math)
#define GCMX_TX2_BUF 1
#endif
#ifndef GCMX_TX2_PROBE_NOX
#define GCMX_TX2_PROBE_NOX 0
#endif
#ifndef GCMX_TX2_DIAG  // tuning builds only: per-wave phase cycle counters (s_memtime)
#define GCMX_TX2_DIAG 0
#endif
#if GCMX_TX2_DIAG
__device__ unsigned long long g_tx2_diag[16][8];  // [wave in block][phase]: cycles summed over blocks
#define TX2_T(i)                                                      \
	do {                                                              \
		const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
		dt_[i] += now_ - tprev_;                                      \
		tprev_ = now_;                                                \
	} while (0)
#else
#define TX2_T(i) \
	do {         \
	} while (0)
#endif
#ifndef GCMX_TX2_GEN2_DEFAULT  // old blocks' share of two generations' rows, percent (0: off; tx2_gen2)
#define GCMX_TX2_GEN2_DEFAULT 64  // 256^3: 0.530-0.540 against 0.547-0.559 ms off, profiles/r6/s
#endif
#ifndef GCMX_TX2_PRIO  // tuning builds only: wave priority while a row's loads are issued (s_setprio)
#define GCMX_TX2_PRIO 0
#endif
#if GCMX_TX2_PRIO
#define TX2_PRIO_HI() __builtin_amdgcn_s_setprio(GCMX_TX2_PRIO)
#define TX2_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#else
#define TX2_PRIO_HI() \
	do {              \
	} while (0)
#define TX2_PRIO_LO() \
	do {              \
	} while (0)
#endif
#ifndef GCMX_TX2_ZPERM  // SIMD partners hold neighbouring z blocks (512^3: 3.548-3.570 against 3.572-3.589 ms, profiles/r6/w)
#define GCMX_TX2_ZPERM 1
#endif
#ifndef GCMX_TX2_BLKT  // tuning builds only: per-wave start / end times (s_memrealtime, 100 MHz) and the
#define GCMX_TX2_BLKT 0  // CU of every block of the last k_step_tx2 launch (gcmx_diag_blk*)
#endif
#if GCMX_TX2_BLKT
constexpr int kBlkMax = 8192;
__device__ unsigned long long g_tx2_blk[kBlkMax][8][2];  // [block][wave][start, end]
__device__ unsigned g_tx2_hw[kBlkMax];                   // HW_ID of the block's wave 0
#endif

// Timing knobs (A/B builds only; the defaults are the product): per-node face
// maps compiled into the FACES ghosts; face values read from LDS instead of the
// kernel arguments; HET_AB 1 = every material uses the kernel-argument table,
// 2 = also no material-id loads (both give wrong HET results: timing only).
#ifndef GCMX_TX2_FACEMAP
#define GCMX_TX2_FACEMAP 1
#endif
#ifndef GCMX_TX2_FACE_LDS
#define GCMX_TX2_FACE_LDS 0
#endif
#ifndef GCMX_TX2_STNT
#define GCMX_TX2_STNT 1  // non-temporal stores of the new layer
#endif
#ifndef GCMX_TX2_ALT
#define GCMX_TX2_ALT 1  // odd y chunks march down (shared halo rows read at the same time)
#endif
#ifndef GCMX_TX2_NTOUTER
#define GCMX_TX2_NTOUTER 0  // timing knob: the outermost window planes by non-temporal loads
#endif
#ifndef GCMX_TX2_NTLOAD
#define GCMX_TX2_NTLOAD 1  // node-only components by non-temporal loads (+0.4 %, profiles/r4/ab)
#endif
#ifndef GCMX_HET_AB
#define GCMX_HET_AB 0
#endif
#ifndef GCMX_ZS_PAIRS_FIRST  // z split: block order pairs fastest (1) or the parts of a pair adjacent (0)
#define GCMX_ZS_PAIRS_FIRST 1  // an XCD's concurrent blocks then cover twice the consecutive pairs: 1024^3 -1.2 % (profiles/r6/n)
#endif

#ifndef GCMX_TX2_UNROLL  // timing knob: row-loop unroll (5 = the window period: no window moves)
#define GCMX_TX2_UNROLL 1
#endif


// Per-node materials: every lane applies ITS OWN material's table, read from
// the LDS copy with a per-lane address.  (Rounds 3-4 wrapped this in a
// readfirstlane "waterfall" loop, `for (;;) { k = readfirstlane(key); if (key
// == k) { f(k); break; } }`, meant to keep k wave-uniform.  Inside `key == k`
// the compiler replaces k by the lane's own key, after which the loop carries
// nothing uniform and is deleted: every lane runs f once with its own key, all
// lanes active.  With tables read per lane that is still correct (and is what
// the shipped round-4 ISA does: ds_read at a per-lane address, no loop); the
// mid-round-4 variant that also passed the table fields through readfirstlane
// (cb6938f) then broadcast the FIRST lane's table to the whole wave -- wrong
// for every lane of another material (relative L2 0.687 on random material
// ids, green on layered ids where a wave holds one material).  DESIGN.md §3.1.)

// Component held in window slot q of a stage whose window mask is `mask`.
__host__ __device__ constexpr int wcomp(unsigned mask, int q) {
	int n = 0;
	for (int j = 0; j < 9; j++)
		if ((mask >> j) & 1u) {
			if (n == q) return j;
			n++;
		}
	return -1;
}

// The whole time step in one pass with TWO adjacent x planes per thread
// (x, x+1 at one z) -- the default 3-D step for borderSize <= 2, Z <= 512.
//
// Why two planes: the X stages of both nodes read the 2*BS+2 planes
// x-BS .. x+1+BS, i.e. 6*(2*BS+2) + 2*3 loads per two nodes instead of
// 2*(6*(2*BS+1) + 3).  Those x-neighbour re-reads are L2->CU traffic, and that
// traffic, not HBM, bounds the one-plane kernel: tools/xyz_probe.hip measures the
// bare access pattern at 33 loads + 9 stores per node 1.35x slower than the
// compulsory 9 + 9, and at two planes per thread 1.12x.
//
// Arithmetic per node is k_fused_xyz's (pair_update / node_update, reference
// operation order), except that with floor(q) == 0 the X stage's Newton
// differences are shared by the two nodes: with forward differences along x,
//   D0_k = S_k,  Di_k = (D(i-1)_{k+1} - D(i-1)_k) * c_{i-1},
// the +x foot of node m interpolates (S_m + D1_m) + D2_m ... exactly as
// minMaxInterpolate does (EqualDistanceLineInterpolator.hpp:56-71), and the -x
// foot, whose values are S_m, S_{m-1}, ..., has d_i = (-1)^i Di_{m-i}, so
// (S_m - D1_{m-1}) + D2_{m-2} ...: a - b == -(b - a) and (-x) * c == -(x * c)
// in IEEE arithmetic, up to the sign of an exact zero (IEEE-equal, DESIGN.md
// §3.2).  The -x limiter bounds of node x+1 are the +x bounds of node x.
//
// Schedule (each choice measured A/B on MI355X): registers hold
// the two Y windows; the node-only Y components of rows y..y+BS (read back by
// the same thread only) live in an LDS ring; the Z exchange is one LDS buffer
// per node with two barriers per row; the first two load pairs of the next row
// are issued before the Z stage, each node's 9 stores right after its own Z
// stage, the last pair and the node-only loads when the X stage starts.  One
// 512-thread block per CU (2 waves/SIMD, <= 256 VGPRs).
//
// FACES: uniform cubic border conditions on the y/z faces (FaceBC): the ghost
// rows of the Y stage and the ghost columns of the Z stage are the mirrored
// inner X / Y results with the overridden components set to -inner + 2 f(t)
// (BorderConditions.hpp:94-114, applied to the intermediate layers as
// Engine::nextTimeStep does before each stage, Engine.cpp:90-121).  Only the
// window components of those ghosts are ever read, so they are all that is
// formed.  Requires Y, Z >= 2*BS+2 (the mirrored rows are inner rows) and no
// PRESSURE condition on a y/z face (its trace needs the node-only components);
// x faces are filled in memory before the launch (k_face_fill).
// Without FACES, y/z ghosts of both layers must be zero.
//
// If the launch has an odd number of planes the last thread's second node is
// computed from clamped (valid) planes and not stored.
//
// HET: per-node materials (heterogeneous media, TestEngine.cpp:139-296's layers).
// Every node's stages use its own material's tables mtab[mat[node]] (per material
// the three axes' tables are identical and floor(q) = 0, checked on the host), as
// GridCharacteristicMethod::stage takes each node's own matrices.  The tables are
// read per lane from their LDS copy; where the two nodes of a lane differ in
// material, their X stages run without the shared differences (pair_update per
// node).
//
// ZS (z split, Z = nz * ZT > 512, uniform medium, no faces): a z row no longer
// fits one block's register windows (two planes x 1024 z x 6 components x 5 rows
// of fp64 = 94 % of a CU's register file), so each row is cut into nz parts of
// ZT lanes, one block each.  A part's Z stage is exact except in the BS lanes
// next to a cut, which need the other part's Y results: those lanes do not
// store, and k_zseam recomputes the X and Y stages of the 4*BS columns around
// each cut and stores their Z stage after the launch (1024^3: 8 of 1024 columns).
// (Handing the cut lanes' Y results over through memory instead cost 25 %: those
// lanes' extra stores sit in the vmcnt queue the row-ahead loads are waited on
// with, profiles/r6/h.)
template <int BS, int ZT, bool KF0, bool UNI, bool FACES, bool HET, bool ZS = false>
__global__ __launch_bounds__(ZT, GCMX_TX2_MINWAVES) void k_step_tx2(
    const double* __restrict__ in, double* __restrict__ outl, Geo g, IsoAxis AX, IsoAxis AY_,
    IsoAxis AZ_, int x0, int chunk, int nplanes, int xb0, int nplanesb, FaceBC fb,
    const IsoAxis* __restrict__ mtab, const uint8_t* __restrict__ mat) {
	static_assert(!HET || (KF0 && UNI), "heterogeneous step: floor(q) = 0, Z == ZT, equal axes");
	static_assert(!ZS || (UNI && !HET), "z split: uniform medium");
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
	// NB: Z == ZT, a multiple of 64.  Each wave keeps its own Y results in a region
	// of 64 + 2 BS slots; only the BS edge values per side cross to the neighbour
	// waves, through a two-row ring `eg` and a per-wave row counter `rdy` (no block
	// barrier: the waves of a block drift apart and overlap their memory phases).
	constexpr bool NB = UNI && GCMX_TX2_NB;
	constexpr int NW = ZT / 64;
	constexpr int RW = 64 + 2 * BS;
	static_assert(!NB || ZT % 64 == 0, "NB needs whole waves");
	constexpr bool ZS2 = GCMX_TX2_ZS2 < 0 ? !NB : GCMX_TX2_ZS2 != 0;
	__shared__ double zl[NB ? 1 : 2][NB ? 1 : NWZ][NB ? 1 : LW];  // Y results of both nodes (Z stage input)
	__shared__ double rg[NB ? NW : 1][NB ? 2 : 1][NB ? NWZ : 1][NB ? RW : 1];
	__shared__ double eg[NB ? 2 : 1][NB ? NW : 1][2][NB ? 2 : 1][NB ? NWZ : 1][BS];  // [row&1][wave][side][node][comp][k]
	__shared__ int rdy[NB ? NW : 1];                                               // last row whose edges are in eg
	__shared__ double cl[BS + 1][2][NCY][ZT];  // node-only Y components, rows y..y+BS (ring)
	// HET: every material's tables in LDS (<= kHetMaxMaterials, host-checked).  A
	// global (or flat: LDS-or-global) table load in the row loop would count in
	// vmcnt, and waiting for it would wait for every row-ahead load issued before
	// it -- the software pipeline collapses (measured: HET 256^3 +34 %).
	__shared__ IsoAxis hlds[HET ? kHetMaxMaterials : 1];
	__shared__ double hode[HET ? kHetMaxMaterials : 1];  // HET: folded ODE factor per material
	__shared__ double flds[FACES && GCMX_TX2_FACE_LDS ? 4 : 1][9];  // 2 f(t) of the y/z faces

#if GCMX_TX2_ZPERM
	// z blocks of 64 columns dealt so that the two waves sharing a SIMD (w and
	// w + 4 of a 512-lane block) hold neighbouring z blocks 2w and 2w + 1
	const int z = [] {
		int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
		if constexpr (ZT == 512) w = w < 4 ? 2 * w : 2 * (w - 4) + 1;
		return w * 64 + (int)(threadIdx.x & 63);
	}();
#else
	const int z = threadIdx.x;
#endif
#if GCMX_TX2_BLKT
	const unsigned long long blk_t0_ = __builtin_amdgcn_s_memrealtime();
#endif
	const int Y = g.sizes[1], Z = g.sizes[2];
	int x, yb, ye, xbeg, xend;
	bool rev;  // this block marches its rows downwards (odd chunks, GCMX_TX2_ALT)
	int zp = 0;                                    // ZS: this block's part of the z row
	const int nz = ZS ? g.sizes[2] / ZT : 1;
	{  // XCD-aware chunk-major block order (see k_fused_xyz) over the plane pairs of
	   // range A [x0, x0 + nplanes), then range B [xb0, xb0 + nplanesb) (may be empty).
	   // Pairs are GLOBAL: (2k, 2k+1) in the global x index g.gx0 + x, so a range
	   // starting at an odd global plane begins with a pair whose first node is not
	   // ours.  The two nodes of a pair run different (contracted, in the FMA build)
	   // operation sequences, so global pairing keeps every node's sequence, and with
	   // it every bit, independent of how the grid is cut into slabs or bodies.
		const int pa = (g.gx0 + x0) & 1, pb = (g.gx0 + xb0) & 1;
		const int npa = (nplanes + pa + 1) / 2;
		const int npair = npa + (nplanesb > 0 ? (nplanesb + pb + 1) / 2 : 0);
		const int T = (int)gridDim.x, b = (int)blockIdx.x;
		int p = xcd_order(b, T);
		if constexpr (ZS && !GCMX_ZS_PAIRS_FIRST) {  // the parts of one (pair, chunk) are neighbours in the order
			zp = p % nz;
			p /= nz;
		}
		int q = p % npair;
		int cidx = p / npair;  // chunk index
		if (!ZS && chunk < 0) {
			// Two generations (tx2_gen2): the launch is exactly two resident blocks per
			// CU, and the first block dispatched to a CU (blocks [0, T/2)) runs ahead of
			// its younger neighbour (oldest-first issue): old blocks take chunks of
			// `co` rows, young ones `cy`.  Per generation, XCD k's blocks take the
			// k-th contiguous run of (pair, chunk slot s) positions, pairs fastest;
			// an old block runs chunk s, a young one chunk ncg + s.
			const int co = (-chunk) & 0xFFFF, half = T >> 4;
			const int j = b >> 3, gen = j >= half ? 1 : 0;
			const int G = (b & 7) * half + (j - gen * half);
			const int ncg = (T >> 1) / npair;  // chunks per generation
			q = G % npair;
			cidx = G / npair + gen * ncg;
			const int cy = (-chunk) >> 16;
			auto start = [&](int c) { return c <= ncg ? c * co : ncg * co + (c - ncg) * cy; };
			yb = start(cidx);
			ye = min(start(cidx + 1), Y);  // the host makes ncg (co + cy) == Y
		}
		x = q < npa ? x0 - pa + 2 * q : xb0 - pb + 2 * (q - npa);
		xbeg = q < npa ? x0 : xb0;
		xend = q < npa ? x0 + nplanes : xb0 + nplanesb;
		if constexpr (ZS && GCMX_ZS_PAIRS_FIRST) {  // pairs fastest, then parts, then chunks
			zp = cidx % nz;
			cidx /= nz;
		}
		if (ZS || chunk > 0) {
			yb = cidx * chunk;
			ye = min(yb + chunk, Y);
		}
		rev = GCMX_TX2_ALT && (cidx & 1);
	}
	const bool one = x >= xbeg;  // node x is ours (else only x + 1 is)
	const bool two = x + 1 < xend;
	const bool live = UNI || z < Z;
	const int zc = live ? z : Z - 1;
	const unsigned stx = (unsigned)g.stride[0];
	const unsigned sty = (unsigned)g.stride[1];
	// plane bases at this block's plane x (SGPRs), offsets relative to them:
	// 32-bit whatever the layer's size (onepass_layout_ok)
	const long long pbase = (long long)x * g.stride[0];
	const unsigned plane = (unsigned)g.origin;  // node (x, 0, 0) from the bases
	const unsigned zo = live ? (unsigned)z : (unsigned)Z;
	// Memory accessors.  ldx(j, k, r): component j of plane x - BS + k (the last
	// plane clamped when x + 1 is not ours), row r, this lane's column;
	// stz(c, t, y, v): component c of node (x + t, y) of the output layer.
#if GCMX_TX2_BUF
	const Planes src(in + pbase, g.cs);
	const PlanesW out_p(outl + pbase, g.cs);
	const unsigned zpart = ZS ? (unsigned)(zp * ZT) : 0u;      // ZS: first column of this part
	const int zg = (int)zpart + zc;                            // the lane's column in the row
	const unsigned lv = (zpart + (unsigned)zc) * 8u, sv = (zpart + zo) * 8u;  // per-lane byte offsets
	const unsigned pxm = plane - (unsigned)BS * stx;      // plane x - BS, row 0, column 0
	auto ldx = [&](int j, int k, int r) {
#if GCMX_TX2_PROBE_NOX  // timing probe only (wrong results): x-neighbour loads re-read the own planes
		k = k < BS ? BS : (k > BS + 1 ? BS + 1 : k);
#endif
		// planes outside the valid range (x - BS when x is not ours, x + 1 + BS when
		// x + 1 is not ours) are read by the discarded node only: clamp them
		const int d = (k == WX - 1 && !two) ? 2 * BS : (k == 0 && !one) ? 1 : k;
		if (GCMX_TX2_NTOUTER && (k == 0 || k == WX - 1))
			return ld_nt_b(src, j, opaque_u32(lv + (pxm + (unsigned)d * stx + (unsigned)r * sty) * 8u));
		return ld_b(src, j, opaque_u32(lv + (pxm + (unsigned)d * stx + (unsigned)r * sty) * 8u));
	};
	// the node-only components of the own planes: read once, by this lane only
	auto ldc = [&](int j, int k, int r) {
		if constexpr (!GCMX_TX2_NTLOAD) return ldx(j, k, r);
		const int d = (k == WX - 1 && !two) ? 2 * BS : (k == 0 && !one) ? 1 : k;
		return ld_nt_b(src, j, opaque_u32(lv + (pxm + (unsigned)d * stx + (unsigned)r * sty) * 8u));
	};
	auto stz = [&](int c, int t, int y, double v) {
		const unsigned o = opaque_u32(sv + (plane + (unsigned)t * stx + (unsigned)y * sty) * 8u);
		if constexpr (GCMX_TX2_STNT) st_nt_b(out_p, c, o, v);
		else st_b(out_p, c, o, v);
	};
#else
	const unsigned base = plane + zc;
	const Planes src(in + pbase, g.cs);
	const PlanesW out_p(outl + pbase, g.cs);
	auto ldx = [&](int j, int k, int r) {
		const int d = (k == WX - 1 && !two) ? BS : (k == 0 && !one) ? 1 - BS : k - BS;
		return src.ld(j, base + (unsigned)r * sty + (unsigned)d * stx);
	};
	auto ldc = [&](int j, int k, int r) { return ldx(j, k, r); };
	auto stz = [&](int c, int t, int y, double v) { out_p.st_nt(c, plane + (unsigned)y * sty + zo + (unsigned)t * stx, v); };
#endif
	// per-material table k (the lane's own material), from the LDS copy made at
	// kernel start.  Measured alternatives: scalar loads through
	// the constant address space spill VGPRs; separate one-table / two-table X
	// paths double the X stage's code; both are slower.
	auto mt = [&](unsigned k) -> const IsoAxis& {
		if constexpr (GCMX_HET_AB >= 1) return AX;
		return hlds[k];
	};
	auto two_v = [&](int f, int j) -> double {
		if constexpr (FACES && GCMX_TX2_FACE_LDS) return flds[f][j];
		return fb.two_v[f][j];
	};
	// The condition of face f at node x + t (pos = the node's z on y faces, its y
	// on z faces), resolved once per node: the overridden components and their
	// 2 f(t) (components in `need` only).  A face with a per-node map (partial
	// faces) takes the face node's own condition; none: the ghost stays 0.
	struct GhostRule {
		unsigned mask;
		bool none;
		double two[9];
	};
	auto ghost_rule = [&](int f, int t, int pos, unsigned need) -> GhostRule {
		GhostRule r;
		r.none = false;
		if (GCMX_TX2_FACEMAP && fb.map[f]) {
			const int xx = (t == 1 && !two) ? x : (t == 0 && !one) ? x + 1 : x + t;
			const unsigned c = fb.map[f][(size_t)xx * (f < 2 ? Z : Y) + pos];
			r.none = c == kNoFaceCond;
			const FaceCond& fc = fb.conds[r.none ? 0u : c];
			r.mask = r.none ? 0u : fc.mask;
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((need >> j) & 1u) r.two[j] = r.none ? 0.0 : fc.two_v[j];
		} else {
			r.mask = fb.mask[f];
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((need >> j) & 1u) r.two[j] = two_v(f, j);
		}
		return r;
	};
	// ghost value of component j: -inner + 2 f(t) if overridden, else the mirror
	auto ghost = [](const GhostRule& r, int j, double v) -> double {
		return r.none ? 0.0 : ((r.mask >> j) & 1u) ? -v + r.two[j] : v;
	};

	const int wv = z >> 6, ln = z & 63;  // wave in block, lane
	// ZS: lanes whose Z stage needs the neighbouring part (k_zseam stores them)
	const bool seam_own = ZS && ((zp > 0 && z < BS) || (zp < nz - 1 && z >= ZT - BS));
	if constexpr (NB) {  // zero halos (z ghosts stay zero without a z face); counters
		if (ln < BS || ln >= 64 - BS) {
			const int hs = ln < BS ? ln : ln + 2 * BS;
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int q = 0; q < NWZ; q++) rg[wv][t][q][hs] = 0.0;
		}
		if (z < NW) rdy[z] = -1;  // rows published, counted in marching order
		__syncthreads();
	} else if (z < 2 * BS) {
		const int gslot = (z < BS) ? z : (Z + z);
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int q = 0; q < NWZ; q++) zl[t][q][gslot] = 0.0;
	}

	typedef double PairWin[2][WX];  // [vel/sig][plane]
	auto pair_load = [&](auto PC, PairWin& w, int r) {
		constexpr int P = decltype(PC)::value;
#pragma unroll
		for (int k = 0; k < WX; k++) {
			w[0][k] = ldx(pair_vel(0, P), k, r);
			w[1][k] = ldx(pair_sig(0, P), k, r);
		}
	};
	// Rows 2P, 2P+1 of r = diag(U * V) for both nodes; A0 / A1: the nodes' tables
	// (`same`: one table, the shared-difference form).
	auto pair_rows = [&](auto PC, const PairWin& w, double (&rr)[2][9], const IsoAxis& A0, const IsoAxis& A1,
	                     bool same) {
		constexpr int P = decltype(PC)::value;
		if (KF0 && !same) {  // HET, two materials in the lane: per node, no shared differences
#pragma unroll
			for (int t = 0; t < 2; t++)
				pair_update<0, BS, true, P>(
				    t ? A1 : A0, [&](int j, int o) { return j == pair_vel(0, P) ? w[0][t + BS + o] : w[1][t + BS + o]; },
				    rr[t][2 * P], rr[t][2 * P + 1]);
		} else if constexpr (KF0 && !GCMX_LAGRANGE) {
			const IsoAxis& AS = A0;  // one table for both nodes
			const double* c = (P == 0) ? AS.c1 : AS.c2;
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
#pragma unroll
				for (int t = 0; t < 2; t++) {
					const int m = t + BS;
					double a = D[0][m], b = D[0][m];
#pragma unroll
					for (int i = 1; i <= BS; i++) {
						a += D[i][m];
						b = (i % 2) ? b - D[i][m - i] : b + D[i][m - i];
					}
					// limiter segments (m, m+1) and (m, m-1): the median form (common.hpp
					// vlimit) takes three ops per foot, less than sharing the segment
					// bounds of node 0's +x foot with node 1's -x foot (2 + 2 per foot)
					ip[v][t] = vlimit(a, D[0][m], D[0][m + 1]);
					im[v][t] = vlimit(b, D[0][m], D[0][m - 1]);
				}
			}
#pragma unroll
			for (int t = 0; t < 2; t++) {
				rr[t][2 * P] = RowSum<0, false, 2 * P>::go(
				    AS, [&](int j) { return j == pair_vel(0, P) ? im[0][t] : im[1][t]; }, 0.0, true);
				rr[t][2 * P + 1] = RowSum<0, false, 2 * P + 1>::go(
				    AS, [&](int j) { return j == pair_vel(0, P) ? ip[0][t] : ip[1][t]; }, 0.0, true);
			}
		} else {
#pragma unroll
			for (int t = 0; t < 2; t++)
				pair_update<0, BS, KF0, P>(
				    t ? A1 : A0, [&](int j, int o) { return j == pair_vel(0, P) ? w[0][t + BS + o] : w[1][t + BS + o]; },
				    rr[t][2 * P], rr[t][2 * P + 1]);
		}
	};
	auto sched_fence = [] { __builtin_amdgcn_sched_barrier(0); };
	using P0 = std::integral_constant<int, 0>;
	using P1 = std::integral_constant<int, 1>;
	using P2 = std::integral_constant<int, 2>;
	// X-stage inputs issued ahead of the X stage: load pairs 0 and 1.
	struct XPre {
		PairWin a, b;
	};
	auto cv_load = [&](double (&cv)[2][9], int r) {
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int j = 0; j < 9; j++)
				if ((CMX >> j) & 1u) cv[t][j] = ldc(j, BS + t, r);
	};
	auto x_load_ahead = [&](XPre& pre, int r) {
		pair_load(P0{}, pre.a, r);
		pair_load(P1{}, pre.b, r);
	};
	// X stage of row r for both nodes: pair 2 and the node-only components are
	// issued first, then the pairs are consumed in order.
	// material of node (x + t, r) (HET; rows outside [0, Y) take row Y-1's: their
	// X results come from zero ghost rows or are replaced by a face's mirror)
	auto mat_of = [&](int t, int r) -> unsigned {
		const int xx = (t == 1 && !two) ? x : (t == 0 && !one) ? x + 1 : x + t;
		const int rr_ = r < 0 ? 0 : (r < Y ? r : Y - 1);
		return mat[((size_t)xx * Y + rr_) * Z + z];
	};
	auto x_compute = [&](const XPre& pre, const PairWin& wc, const double (&cv)[2][9], double (&xr)[2][9],
	                     const IsoAxis& A0, const IsoAxis& A1, bool same) {
		double rr[2][9], n0[2][9];
		pair_rows(P0{}, pre.a, rr, A0, A1, same);
		pair_rows(P1{}, pre.b, rr, A0, A1, same);
		sched_fence();
		pair_rows(P2{}, wc, rr, A0, A1, same);
#pragma unroll
		for (int t = 0; t < 2; t++) {
			n0[t][pair_vel(0, 0)] = pre.a[0][t + BS];
			n0[t][pair_sig(0, 0)] = pre.a[1][t + BS];
			n0[t][pair_vel(0, 1)] = pre.b[0][t + BS];
			n0[t][pair_sig(0, 1)] = pre.b[1][t + BS];
			n0[t][pair_vel(0, 2)] = wc[0][t + BS];
			n0[t][pair_sig(0, 2)] = wc[1][t + BS];
		}
		sched_fence();
#pragma unroll
		for (int t = 0; t < 2; t++) {
			const IsoAxis& A = t ? A1 : A0;
			center_update<0>(A, [&](int j) { return ((WMX >> j) & 1u) ? n0[t][j] : cv[t][j]; }, rr[t]);
			u1_apply<0>(A, rr[t], xr[t]);
		}
	};
	// HET: the two nodes' materials of row r as one key (node x in bits 0-7)
	auto key_of = [&](int r) -> unsigned {
		if constexpr (GCMX_HET_AB >= 2) return 0u;
		return mat_of(0, r) | (mat_of(1, r) << 8);
	};
	// key: key_of(r), loaded ahead by the caller (HET)
	auto x_stage = [&](const XPre& pre, int r, double (&xr)[2][9], unsigned key) {
		PairWin wc;
		double cv[2][9];
		TX2_PRIO_HI();
		pair_load(P2{}, wc, r);
		cv_load(cv, r);
		TX2_PRIO_LO();
		sched_fence();
		if constexpr (HET) {
			const unsigned m0 = key & 255u, m1 = key >> 8;
			x_compute(pre, wc, cv, xr, mt(m0), mt(m1), m0 == m1);
		} else {
			x_compute(pre, wc, cv, xr, AX, AX, true);
		}
	};

	double win[2][NWY][W];
	// HET: material keys of the window's rows (slot k: row y - BS + k), each loaded
	// once, one row ahead of its X stage, and reused by that row's Y and Z stages
	unsigned hk[W];
#pragma unroll
	for (int k = 0; k < W; k++) hk[k] = 0;
	if constexpr (HET) {  // tables into LDS (het tables are allocated for 256 materials)
		for (int i = z; i < kHetMaxMaterials * (int)(sizeof(IsoAxis) / 4); i += ZT)
			reinterpret_cast<unsigned*>(hlds)[i] = reinterpret_cast<const unsigned*>(mtab)[i];
		if (fb.ode_on && fb.ode_f && z < kHetMaxMaterials) hode[z] = fb.ode_f[z];
	}
	if constexpr (FACES && GCMX_TX2_FACE_LDS) {
#pragma unroll
		for (int c = 0; c < 36; c++)
			if (z == c) flds[c / 9][c % 9] = fb.two_v[c / 9][c % 9];
	}
	if constexpr (HET || (FACES && GCMX_TX2_FACE_LDS)) __syncthreads();
	// The row march, in either direction (REV: from the chunk's last row down).
	// Odd chunks march down, so the halo rows two adjacent chunks both compute
	// the X stage of are read by both blocks at the same time -- both at the
	// start or both at the end of their march -- and the second read hits the
	// caches (a forward-only march reads them at opposite ends of the launch:
	// 256^3, 64-row chunks, 1.13x the compulsory reads from HBM).
	auto run = [&](auto RV) {
	constexpr bool REV = decltype(RV)::value;
	constexpr int S = REV ? -1 : 1;
	// node-only Y components: ring slot of row r; per-lane pointer with the
	// (node, component) part as a constant LDS offset
	auto cl_at = [&](int r) { return &cl[(r + 2 * BS + 2) % (BS + 1)][0][0][z]; };
	// row r's X result enters window slot `slot`; its node-only components go to the ring
	auto push = [&](const double (&xr)[2][9], int slot, int r) {
		double* cp = cl_at(r);
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int j = 0; j < 9; j++) {
				if ((WMY >> j) & 1u) win[t][wslot(WMY, j)][slot] = xr[t][j];
				if ((CMY >> j) & 1u) cp[(t * NCY + wslot(CMY, j)) * ZT] = xr[t][j];
			}
	};
	// window slot k := ghost of face f mirrored from window slot ks (a runtime
	// index, resolved by compile-time selects; rare path)
	auto mirror_slot = [&](int k, int ks, int f) {
#pragma unroll
		for (int t = 0; t < 2; t++) {
			const GhostRule gr = ghost_rule(f, t, zg, WMY);
#pragma unroll
			for (int q = 0; q < NWY; q++) {
				double v = 0.0;
#pragma unroll
				for (int kk = 0; kk < W; kk++)
					if (kk == ks) v = win[t][q][kk];
				const double gv = ghost(gr, wcomp(WMY, q), v);
#pragma unroll
				for (int kk = 0; kk < W; kk++)
					if (kk == k) win[t][q][kk] = gv;
			}
		}
	};
	// prologue: X results of rows y0-BS .. y0+BS (rows < 0 or >= Y are ghosts);
	// window slot k holds row y + S*(k - BS) of the current row y
	const int y0 = REV ? ye - 1 : yb;
#pragma unroll
	for (int k = 0; k < W; k++) {
		const int r = y0 + S * (k - BS);
		double xr[2][9];
		if (r >= 0 && r < Y) {
			XPre pre;
			if constexpr (HET) hk[k] = key_of(r);
			x_load_ahead(pre, r);
			x_stage(pre, r, xr, hk[k]);
		} else {
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++) xr[t][j] = 0.0;
		}
		push(xr, k, r);  // the first BS rows are overwritten in the ring by the last BS
	}
	if constexpr (FACES) {  // ghost rows of the prologue window: mirrors of inner rows
		if (fb.on & 3u) {
#pragma unroll
			for (int k = 0; k < W; k++) {
				const int r = y0 + S * (k - BS);
				const int f = r < 0 ? 0 : 1, ks = BS + S * ((r < 0 ? -r : 2 * (Y - 1) - r) - y0);
				if ((r < 0 || r >= Y) && ((fb.on >> f) & 1u) && ks >= 0 && ks < W) mirror_slot(k, ks, f);
			}
		}
	}
	auto clamp_row = [&](int r) {  // rows beyond the ghost rows (their X results go unused)
		if constexpr (REV) return r > -BS ? r : -BS;
		return r < Y + BS - 1 ? r : Y + BS - 1;
	};

#if GCMX_TX2_DIAG
	unsigned long long dt_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
	// Y stage of row y for both nodes (window + node-only ring)
	auto y_stage = [&](int y, double (&yv)[2][9]) {
		const double* cp = cl_at(y);
#pragma unroll
		for (int t = 0; t < 2; t++) {
			auto go = [&](const IsoAxis& A) {
				node_update<1, BS, KF0>(
				    A, [&](int j, int o) { return win[t][wslot(WMY, j)][BS + S * o]; },
				    [&](int j) { return ((WMY >> j) & 1u) ? win[t][wslot(WMY, j)][BS] : cp[(t * NCY + wslot(CMY, j)) * ZT]; },
				    yv[t]);
			};
			if constexpr (HET) go(mt(t ? hk[BS] >> 8 : hk[BS] & 255u));
			else go(AY);
		}
	};
	// z ghosts of row y (FACES): lanes 1..BS form the z- face's ghost columns,
	// lanes Z-1-BS..Z-2 the z+ face's, put(side, node, window slot, value) -- one
	// divergent region per face and row, entered only by the waves holding those
	// lanes, one condition lookup per node
	auto z_ghosts = [&](int y, const double (&yv)[2][9], auto&& put) {
		const int wu = __builtin_amdgcn_readfirstlane(z >> 6);
#pragma unroll
		for (int side = 0; side < 2; side++) {
			// ZS: the z- face lies in the first part, the z+ face in the last, at
			// lanes of that part (Zl: the part's row length)
			const int Zl = ZS ? ZT : Z;
			if (ZS && (side ? zp != nz - 1 : zp != 0)) continue;
			const int lo = side ? Zl - 1 - BS : 1, hi = side ? Zl - 2 : BS;
			if (!((fb.on >> (2 + side)) & 1u) || wu * 64 > hi || wu * 64 + 63 < lo) continue;
			if (z < lo || z > hi) continue;
#pragma unroll
			for (int t = 0; t < 2; t++) {
				const GhostRule gr = ghost_rule(2 + side, t, y, WMZ);
#pragma unroll
				for (int j = 0; j < 9; j++)
					if ((WMZ >> j) & 1u) put(side, t, wslot(WMZ, j), ghost(gr, j, yv[t][j]));
			}
		}
	};
	// hand the Y results of row y to the Z stage: NB, own region + edge ring +
	// counter; otherwise the block buffer between two barriers
	auto publish = [&](int it, int y, const double (&yv)[2][9]) {
		const int es = it & 1;  // NB: edge ring slot of this row (it: the row's place in the march)
		if constexpr (NB) {
			// this lane's edge slot (lanes < BS: left side, >= 64 - BS: right side);
			// (node, component) as a constant LDS offset
			double* egp = ln < BS ? &eg[es][wv][0][0][0][ln] : &eg[es][wv][1][0][0][ln - (64 - BS)];
			const bool edge = ln < BS || ln >= 64 - BS;
			asm volatile("" ::: "memory");  // after the previous row's Z-stage reads of rg
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++)
					if ((WMZ >> j) & 1u) {
						const int q = wslot(WMZ, j);
						rg[wv][t][q][BS + ln] = yv[t][j];
						if (edge) egp[(t * NWZ + q) * BS] = yv[t][j];
					}
			if constexpr (FACES)  // z ghosts: wave 0's left halo, the last wave's right halo
				z_ghosts(y, yv, [&](int side, int t, int q, double v) {
					if (side == 0) rg[0][t][q][BS - z] = v;
					else rg[NW - 1][t][q][BS + 2 * ((ZS ? ZT : Z) - 1) - z - 64 * (NW - 1)] = v;
				});
			// edges in LDS before the counter says so (LDS only: global memory keeps flowing)
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			__hip_atomic_store(&rdy[wv], it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		} else {
			__syncthreads();  // every wave has finished reading zl (previous row's Z stage)
#pragma unroll
			for (int t = 0; t < 2; t++)
#pragma unroll
				for (int j = 0; j < 9; j++)
					if ((WMZ >> j) & 1u) {
						const int q = wslot(WMZ, j);
						if constexpr (FACES) {
							// idle lanes leave the z ghost slots to the face (or their zero)
							if (UNI || z < Z || z >= Z + BS) zl[t][q][BS + z] = live ? yv[t][j] : 0.0;
						} else {
							zl[t][q][BS + z] = live ? yv[t][j] : 0.0;
						}
					}
			if constexpr (FACES)
				z_ghosts(y, yv, [&](int side, int t, int q, double v) {
					if (side == 0) zl[t][q][BS - z] = v;
					else zl[t][q][BS + 2 * (Z - 1) - z] = v;
				});
			__syncthreads();
		}
	};
	// NB: wait for the neighbour waves' edges of row y, copy them into the own halo slots
	auto collect = [&](int it) {
		if constexpr (NB && NW > 1) {
			const int es = it & 1;
			for (;;) {
				const int a = wv > 0 ? __hip_atomic_load(&rdy[wv - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : it;
				const int b =
				    wv < NW - 1 ? __hip_atomic_load(&rdy[wv + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : it;
				if (__builtin_amdgcn_readfirstlane(min(a, b)) >= it) break;
				if constexpr (GCMX_TX2_SLEEP > 0) __builtin_amdgcn_s_sleep(GCMX_TX2_SLEEP);
			}
			asm volatile("" ::: "memory");
			if (ln < BS && wv > 0) {
#pragma unroll
				for (int t = 0; t < 2; t++)
#pragma unroll
					for (int q = 0; q < NWZ; q++) rg[wv][t][q][ln] = eg[es][wv - 1][1][t][q][ln];
			}
			if (ln >= 64 - BS && wv < NW - 1) {
#pragma unroll
				for (int t = 0; t < 2; t++)
#pragma unroll
					for (int q = 0; q < NWZ; q++) rg[wv][t][q][ln + 2 * BS] = eg[es][wv + 1][0][t][q][ln - (64 - BS)];
			}
			asm volatile("" ::: "memory");
		}
	};
	// Z stage of node t of row y and its 9 stores
	auto z_stage_store = [&](int t, int y, const double (&yv)[2][9]) {
		double zv[9];
		auto go = [&](const IsoAxis& A) {
			if constexpr (NB)
				node_update<2, BS, KF0>(
				    A, [&](int j, int o) { return rg[wv][t][wslot(WMZ, j)][BS + ln + o]; },
				    [&](int j) { return ((WMZ >> j) & 1u) ? rg[wv][t][wslot(WMZ, j)][BS + ln] : yv[t][j]; }, zv);
			else
				node_update<2, BS, KF0>(
				    A, [&](int j, int o) { return zl[t][wslot(WMZ, j)][BS + z + o]; },
				    [&](int j) { return ((WMZ >> j) & 1u) ? zl[t][wslot(WMZ, j)][BS + z] : yv[t][j]; }, zv);
		};
		if constexpr (HET) go(mt(t ? hk[BS] >> 8 : hk[BS] & 255u));
		else go(AZ);
		if (fb.ode_on) {  // MaxwellViscosityOde: sigma *= exp(-tau / tau0), the stored product (Ode.hpp:34-35)
			double f = fb.ode;
			if constexpr (HET)  // the node's own material's factor
				if (fb.ode_f) f = hode[t ? hk[BS] >> 8 : hk[BS] & 255u];
#pragma unroll
			for (int c = 3; c < 9; c++) zv[c] = zv[c] * f;
		}
		if ((t == 0 ? one : two) && !(ZS && seam_own)) {
#pragma unroll
			for (int c = 0; c < 9; c++) stz(c, t, y, live ? zv[c] : 0.0);
		}
	};
	// X stage of row y+S*(BS+1) -> window slot W-1 (ghost rows: zero, or a face's mirror)
	auto x_enter = [&](int y, const XPre& pre, unsigned kn) {
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int q = 0; q < NWY; q++)
#pragma unroll
				for (int o = 0; o < W - 1; o++) win[t][q][o] = win[t][q][o + 1];
		if constexpr (HET) {
#pragma unroll
			for (int o = 0; o < W - 1; o++) hk[o] = hk[o + 1];
			hk[W - 1] = kn;
		}
		double xr[2][9];
		sched_fence();
		const int r = y + S * (BS + 1);
		x_stage(pre, clamp_row(r), xr, kn);
		push(xr, W - 1, r);
		sched_fence();
		if constexpr (FACES) {
			const int f = r < 0 ? 0 : 1;
			if ((r < 0 || r >= Y) && ((fb.on >> f) & 1u)) {  // slot of the mirrored row in the next row's window
				const int ks = BS + S * ((r < 0 ? -r : 2 * (Y - 1) - r) - (y + S));
				if (ks >= 0 && ks < W) mirror_slot(W - 1, ks, f);
			}
		}
	};
	auto row = [&](int y, int it) {
		double yv[2][9];
		XPre pre;
		const int rn = clamp_row(y + S * (BS + 1));
		unsigned kn = 0;  // HET: row rn's materials, one row ahead of its X stage
		if constexpr (HET) kn = key_of(rn);
		y_stage(y, yv);
		TX2_T(0);
		publish(it, y, yv);
		TX2_T(2);
		if constexpr (ZS2) {
			sched_fence();
			pair_load(P0{}, pre.a, rn);
			sched_fence();
		} else {  // loads older than this row's stores
			sched_fence();
			TX2_PRIO_HI();
			x_load_ahead(pre, rn);
			TX2_PRIO_LO();
			sched_fence();
		}
		TX2_T(6);
		collect(it);
		TX2_T(4);
#pragma unroll
		for (int t = 0; t < 2; t++) {  // each node's stores right after its Z stage
			if constexpr (ZS2) {
				if (t == 1) {
					sched_fence();
					pair_load(P1{}, pre.b, rn);
					sched_fence();
				}
			}
			z_stage_store(t, y, yv);
		}
		TX2_T(3);
		x_enter(y, pre, kn);
		TX2_T(5);
	};
#if GCMX_TX2_UNROLL > 1
#pragma unroll GCMX_TX2_UNROLL
#endif
	for (int it = 0; it < ye - yb; it++) row(REV ? ye - 1 - it : yb + it, it);
#if GCMX_TX2_BLKT
	if ((threadIdx.x & 63) == 0 && blockIdx.x < (unsigned)kBlkMax && threadIdx.x < 512) {
		const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
		g_tx2_blk[blockIdx.x][threadIdx.x / 64][0] = blk_t0_;
		g_tx2_blk[blockIdx.x][threadIdx.x / 64][1] = t1;
		if (threadIdx.x == 0) g_tx2_hw[blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
	}
#endif
#if GCMX_TX2_DIAG
	if ((threadIdx.x & 63) == 0) {
		const int wv = threadIdx.x / 64;
		for (int i = 0; i < 8; i++) atomicAdd(&g_tx2_diag[wv][i], dt_[i]);
	}
#endif
	};
	if (rev) run(std::true_type{});
	else run(std::false_type{});
}

// The nodes next to the cuts of a z-split step (k_step_tx2<..., ZS>), after it:
// lane (plane, column) of a group of 4*BS lanes holds one of the columns
// cut - 2*BS ... cut + 2*BS - 1 of one x plane and marches y like k_fused_xyz --
// the X stage of the entering row (node_update<0>: the same per-node operations
// as the one-pass step's X stage), the Y stage from its register window -- then
// the Z stage of the middle 2*BS columns from the group's Y results (lane
// shuffles), the folded ODE factor, 9 stores.  Rows: `chunk` per block, the
// 2*BS-row prologue recomputed.  Reads the 4*BS columns' neighbourhoods (mostly
// L2), writes 2*BS columns per cut: at 1024^3 0.4 % of the step's bytes.
//
// FACES: y-face conditions as the one-pass step forms them (FaceBC, uniform or a
// per-node map): a window row outside [0, Y) is the mirrored inner row with the
// condition's components set to -inner + 2 f(t) (BorderConditions.hpp:94-114).
template <int BS, bool KF0, bool FACES>
__global__ __launch_bounds__(256) void k_zseam(const double* __restrict__ in, double* __restrict__ outl, Geo g,
                                                IsoAxis A, int x0, int nplanes, int xb0, int nplanesb, int zt,
                                                int chunk, FaceBC fb) {
	const unsigned ode_on = fb.ode_on;
	const double ode = fb.ode;
	constexpr int NC = 4 * BS, PB = 256 / NC, W = 2 * BS + 1;
	const int Y = g.sizes[1], ncut = g.sizes[2] / zt - 1;
	const int nch = (Y + chunk - 1) / chunk;
	int b = (int)blockIdx.x;
	const int ch = b % nch;
	b /= nch;
	const int cut = b % ncut;
	const int pg = b / ncut;
	const int c = (int)threadIdx.x % NC, xi = pg * PB + (int)threadIdx.x / NC;
	const bool valid = xi < nplanes + nplanesb;
	const int x = !valid ? x0 : xi < nplanes ? x0 + xi : xb0 + (xi - nplanes);
	const int z = (cut + 1) * zt - 2 * BS + c;
	const long long stx = g.stride[0], sty = g.stride[1], cs = g.cs;
	const long long base = g.origin + (long long)x * stx + z;
	const int yb = ch * chunk, ye = min(yb + chunk, Y);
	// X result of row r (rows outside [0, Y): zero ghost rows; beyond them clamped)
	auto xstage = [&](int r, double (&xr)[9]) {
		const int rc = r < -BS ? -BS : (r > Y + BS - 1 ? Y + BS - 1 : r);
		const long long o = base + (long long)rc * sty;
		node_update<0, BS, KF0>(
		    A, [&](int j, int oo) { return in[j * cs + o + oo * stx]; }, [&](int j) { return in[j * cs + o]; }, xr);
	};
	double win[9][W];
	// window slot k := the ghost of y face f mirrored from slot ks (runtime slot
	// indices resolved by compile-time selects, as k_step_tx2's mirror_slot)
	auto mirror = [&](int k, int ks, int f) {
		unsigned mask;
		bool none = false;
		double two[9];
		if (fb.map[f]) {
			const unsigned cnd = fb.map[f][(size_t)x * g.sizes[2] + z];
			none = cnd == kNoFaceCond;
			const FaceCond& fc = fb.conds[none ? 0u : cnd];
			mask = none ? 0u : fc.mask;
#pragma unroll
			for (int j = 0; j < 9; j++) two[j] = none ? 0.0 : fc.two_v[j];
		} else {
			mask = fb.mask[f];
#pragma unroll
			for (int j = 0; j < 9; j++) two[j] = fb.two_v[f][j];
		}
#pragma unroll
		for (int j = 0; j < 9; j++) {
			double v = 0.0;
#pragma unroll
			for (int kk = 0; kk < W; kk++)
				if (kk == ks) v = win[j][kk];
			const double gv = none ? 0.0 : ((mask >> j) & 1u) ? -v + two[j] : v;
#pragma unroll
			for (int kk = 0; kk < W; kk++)
				if (kk == k) win[j][kk] = gv;
		}
	};
#pragma unroll
	for (int k = 0; k < W; k++) {
		double xr[9];
		const int r = yb - BS + k;
		if (r >= 0 && r < Y) xstage(r, xr);
		else
#pragma unroll
			for (int j = 0; j < 9; j++) xr[j] = 0.0;
#pragma unroll
		for (int j = 0; j < 9; j++) win[j][k] = xr[j];
	}
	if constexpr (FACES) {  // ghost rows of the prologue window: mirrors of inner rows
		if (fb.on & 3u) {
#pragma unroll
			for (int k = 0; k < W; k++) {
				const int r = yb - BS + k;
				const int f = r < 0 ? 0 : 1, ks = BS + ((r < 0 ? -r : 2 * (Y - 1) - r) - yb);
				if ((r < 0 || r >= Y) && ((fb.on >> f) & 1u) && ks >= 0 && ks < W) mirror(k, ks, f);
			}
		}
	}
	const bool mine = valid && c >= BS && c < 3 * BS;  // the columns whose Z stage the parts left
	const int lane = (int)(threadIdx.x & 63);
	for (int y = yb; y < ye; y++) {
		double yv[9], zv[9];
		node_update<1, BS, KF0>(A, [&](int j, int o) { return win[j][BS + o]; }, [&](int j) { return win[j][BS]; }, yv);
		// z neighbours: lanes c +- o of the same group (the group never straddles a wave)
		node_update<2, BS, KF0>(
		    A, [&](int j, int o) { return __shfl(yv[j], lane + o, 64); }, [&](int j) { return yv[j]; }, zv);
		if (mine) {
			if (ode_on) {
#pragma unroll
				for (int k = 3; k < 9; k++) zv[k] = zv[k] * ode;
			}
			const long long off = base + (long long)y * sty;
#pragma unroll
			for (int k = 0; k < 9; k++) __builtin_nontemporal_store(zv[k], outl + k * cs + off);
		}
#pragma unroll
		for (int j = 0; j < 9; j++)
#pragma unroll
			for (int k = 0; k < W - 1; k++) win[j][k] = win[j][k + 1];
		double xr[9];
		const int r = y + BS + 1;
		if (r < Y) xstage(r, xr);
		else
#pragma unroll
			for (int j = 0; j < 9; j++) xr[j] = 0.0;
#pragma unroll
		for (int j = 0; j < 9; j++) win[j][W - 1] = xr[j];
		if constexpr (FACES) {  // the entering row is a y+ ghost row: the mirror of an inner row
			if (r >= Y && ((fb.on >> 1) & 1u)) {
				const int ks = BS + (2 * (Y - 1) - r) - (y + 1);
				if (ks >= 0 && ks < W) mirror(W - 1, ks, 1);
			}
		}
	}
}

// ------------------------------------------------------------- launchers --

static bool same_axis(const IsoAxis& p, const IsoAxis& q) {  // bitwise
	static_assert(sizeof(IsoAxis) == 18 * 8 + 2 * 4, "IsoAxis has padding");
	return std::memcmp(&p, &q, sizeof(IsoAxis)) == 0;
}

// The instance a launch runs, as a readable symbol (gcmx_profile_kernel).
template <int BS, int ZT, bool KF0, bool UNI, bool FACES, bool HET, bool ZS = false>
static const char* tx2_name() {
	static const std::string s = "k_step_tx2<" + std::to_string(BS) + ", " + std::to_string(ZT) + ", " +
	                             (KF0 ? "KF0" : "!KF0") + ", " + (UNI ? "UNI" : "!UNI") + ", " +
	                             (FACES ? "FACES" : "!FACES") + (HET ? ", HET" : "") + (ZS ? ", ZS" : "") +
	                             GCMX_FP_TAG + ">";
	return s.c_str();
}
template <int BS, int ZT, bool KF0, bool UNI>
static const char* xyz_name() {
	static const std::string s = "k_fused_xyz<" + std::to_string(BS) + ", " + std::to_string(ZT) + ", " +
	                             (KF0 ? "KF0" : "!KF0") + ", " + (UNI ? "UNI" : "!UNI") + GCMX_FP_TAG + ">";
	return s.c_str();
}

// Rows per block of k_step_tx2 (req > 0 forces a value): the longest chunk of
// the form Y, 512, 256, ..., 16 whose launch still fills >= 90 % of the resident
// block slots (`slots` = CUs x blocks per CU), so one round of blocks covers the
// launch with the fewest 2*BS-row prologues (measured, DESIGN.md §3.1 / §5:
// 512^3 512 rows 4.32 vs 256 rows 4.37 ms; a 60-plane slab interior 64 rows
// 0.54 vs 32 rows 0.56 vs 16 rows 0.60 ms; 256^3 64 rows 0.590 vs 32 / 128 rows
// 0.599 / 0.692 ms).
static int tx2_chunk_for(int Y, int npair, int req, int slots) {
	if (req > 0) return Y <= req ? Y : req;
	for (int t = 1024; t >= 16; t /= 2) {
		const int ch = Y < t ? Y : t;
		if (10LL * npair * ((Y + ch - 1) / ch) >= 9LL * slots) return ch;
	}
	return Y < 16 ? Y : 16;
}

static int device_cus();
// Two generations of rows (k_step_tx2's chunk < 0): when a launch is exactly two
// resident blocks per CU, the block dispatched first to a CU finishes ~25 %
// before its co-resident younger block (256^3: 0.40 against 0.51 ms,
// profiles/r6/r), and the CU runs the rest at half occupancy.  Old blocks then
// take `co` rows and young ones `cy` (co + cy = 2 Y / nchunk; GCMX_TX2_GEN2 =
// the old share in percent, 0 = off).  Returns the kernel's chunk argument.
static int tx2_gen2(int Y, int npair, int chunk, int T, int per_cu) {
	static const int pct = [] {
		const char* e = std::getenv("GCMX_TX2_GEN2");
		return e ? std::atoi(e) : GCMX_TX2_GEN2_DEFAULT;
	}();
	if (pct <= 50 || pct >= 100 || per_cu != 2 || T != 2 * device_cus() || T % 16 || (T / 2) % npair) return chunk;
	const int nchunk = T / npair;
	if (Y % chunk || Y / chunk != nchunk) return chunk;
	const int ncg = nchunk / 2, two = Y / ncg;  // rows of one old + one young chunk
	if (two * ncg != Y) return chunk;
	const int co = (two * pct + 50) / 100, cy = two - co;
	if (cy < 2 * 2 + 1 || co > 0xFFFF) return chunk;
	return -(co | (cy << 16));
}

static int device_cus() {
	static int n = [] {
		int dev = 0, v = 0;
		if (hipGetDevice(&dev) != hipSuccess ||
		    hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
			v = 256;
		return v;
	}();
	return n;
}

// Rows per block (k_fused_xyz): GCMX_XYZ_CHUNK (128) while the launch still has >= 1024 blocks
// (two rounds of the 512 resident blocks, 2 per CU); thinner slabs (multi-GPU
// X slabs, the boundary planes) halve it, down to 16 rows, to keep every CU
// busy.  Each block recomputes 2*BS X rows in its prologue, so a chunk of c
// rows costs (c + 2*BS) / c of the X stage.  `req` > 0 forces a value.
static int xyz_chunk_for(int Y, int nplanes, int req, int start = GCMX_XYZ_CHUNK, int min_blocks = 1024) {
	int chunk = req > 0 ? req : start;
	if (req <= 0)
		while (chunk > 16 && (long long)((Y + chunk - 1) / chunk) * nplanes < min_blocks) chunk /= 2;
	return Y <= chunk ? Y : chunk;
}

// z split (k_step_tx2<BS, P, ..., ZS> + k_zseam): parts of P lanes, uniform
// medium (equal axes, floor(q) = 0); FACES: the y/z face conditions.
template <int BS, int P, bool FACES>
static void launch_zs(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0, int x1, int xb0, int xb1,
                      hipStream_t st, int req_chunk, const FaceBC* fb, const char** kname) {
	const int nz = g.sizes[2] / P, nb = xb1 > xb0 ? xb1 - xb0 : 0;
	const int npair = (x1 - x0 + ((g.gx0 + x0) & 1) + 1) / 2 + (nb > 0 ? (nb + ((g.gx0 + xb0) & 1) + 1) / 2 : 0);
	// 128 rows per block unless asked: 1024^3 35.2 ms against 36.3 (256 rows),
	// 36.6 (64) and 39.0 (1024, the one-round rule of the Z <= 512 step),
	// profiles/r6/e
	const int chunk = req_chunk > 0 ? std::min(req_chunk, g.sizes[1]) : std::min(128, g.sizes[1]);
	const dim3 grid(((g.sizes[1] + chunk - 1) / chunk) * npair * nz);
	const FaceBC none{};
	const FaceBC& f = fb ? *fb : none;
	hipLaunchKernelGGL((k_step_tx2<BS, P, true, true, FACES, false, true>), grid, dim3(P), 0, st, in, out, g, a[0],
	                   a[1], a[2], x0, chunk, x1 - x0, xb0, nb, f, nullptr, nullptr);
	// the cut columns: 256 / (4 BS) planes per block, 64-row chunks
	const int np = (x1 - x0) + nb, pb = 256 / (4 * BS), sch = std::min(64, g.sizes[1]);
	const long long nblk = (long long)((np + pb - 1) / pb) * (nz - 1) * ((g.sizes[1] + sch - 1) / sch);
	hipLaunchKernelGGL((k_zseam<BS, true, FACES>), dim3((unsigned)nblk), dim3(256), 0, st, in, out, g, a[0], x0,
	                   x1 - x0, xb0, nb, P, sch, f);
	*kname = tx2_name<BS, P, true, true, FACES, false, true>();
}

template <int BS, int ZT>
static void launch_xyz_t(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                         int x1, int xb0, int xb1, hipStream_t st, int req_chunk, const FaceBC* fb,
                         const char** kname, const HetMaterials* het) {
	bool kf0 = true;
	for (int s = 0; s < 3; s++) kf0 = kf0 && a[s].kf1 == 0 && a[s].kf2 == 0;
	const bool uni = kf0 && g.sizes[2] == ZT && same_axis(a[0], a[1]) && same_axis(a[0], a[2]);
	if constexpr (BS <= 2 && ZT <= 512) {
		if (GCMX_XYZ_TX2 || fb) {
			const int nb = xb1 > xb0 ? xb1 - xb0 : 0;
			// global pairs (k_step_tx2): a range starting at an odd global plane
			// begins with a half pair
			const int npair = (x1 - x0 + ((g.gx0 + x0) & 1) + 1) / 2 +
			                  (nb > 0 ? (nb + ((g.gx0 + xb0) & 1) + 1) / 2 : 0);
			// resident blocks: 2 waves per SIMD (<= 256 VGPRs), i.e. 512 / ZT per CU
			const int chunk = tx2_chunk_for(g.sizes[1], npair, req_chunk, device_cus() * (512 / ZT));
			const dim3 grid(((g.sizes[1] + chunk - 1) / chunk) * npair);
			const int cparam = req_chunk > 0 ? chunk : tx2_gen2(g.sizes[1], npair, chunk, (int)grid.x, 512 / ZT);
			const FaceBC none{};
			const FaceBC& f = fb ? *fb : none;
			const IsoAxis* mt = het ? het->tab : nullptr;
			const uint8_t* mi = het ? het->ids : nullptr;
			auto go = [&](auto K, const char* name) {
				hipLaunchKernelGGL(K, grid, dim3(ZT), 0, st, in, out, g, a[0], a[1], a[2], x0, cparam, x1 - x0, xb0,
				                   nb, f, mt, mi);
				*kname = name;
			};
			if (het) {  // the caller checked Z == ZT, KF0 and equal axes per material
				if (fb && fb->on) go(k_step_tx2<BS, ZT, true, true, true, true>, tx2_name<BS, ZT, true, true, true, true>());
				else go(k_step_tx2<BS, ZT, true, true, false, true>, tx2_name<BS, ZT, true, true, false, true>());
				return;
			}
			if (fb && fb->on) {
				if (uni) go(k_step_tx2<BS, ZT, true, true, true, false>, tx2_name<BS, ZT, true, true, true, false>());
				else if (kf0) go(k_step_tx2<BS, ZT, true, false, true, false>, tx2_name<BS, ZT, true, false, true, false>());
				else go(k_step_tx2<BS, ZT, false, false, true, false>, tx2_name<BS, ZT, false, false, true, false>());
			} else {
				if (uni) go(k_step_tx2<BS, ZT, true, true, false, false>, tx2_name<BS, ZT, true, true, false, false>());
				else if (kf0) go(k_step_tx2<BS, ZT, true, false, false, false>, tx2_name<BS, ZT, true, false, false, false>());
				else go(k_step_tx2<BS, ZT, false, false, false, false>, tx2_name<BS, ZT, false, false, false, false>());
			}
			return;
		}
	}
	if (xb1 > xb0) {  // k_fused_xyz has no second range: two launches
		launch_xyz_t<BS, ZT>(in, out, g, a, x0, x1, 0, 0, st, req_chunk, fb, kname, het);
		x0 = xb0;
		x1 = xb1;
	}
	const int chunk = xyz_chunk_for(g.sizes[1], x1 - x0, req_chunk);
	const dim3 grid(((g.sizes[1] + chunk - 1) / chunk) * (x1 - x0));
	if (uni) {
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, true, true>), grid, dim3(ZT), 0, st, in, out, g, a[0], a[1],
		                   a[2], x0, chunk, x1 - x0);
		*kname = xyz_name<BS, ZT, true, true>();
	} else if (kf0) {
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, true, false>), grid, dim3(ZT), 0, st, in, out, g, a[0], a[1],
		                   a[2], x0, chunk, x1 - x0);
		*kname = xyz_name<BS, ZT, true, false>();
	} else {
		hipLaunchKernelGGL((k_fused_xyz<BS, ZT, false, false>), grid, dim3(ZT), 0, st, in, out, g, a[0], a[1],
		                   a[2], x0, chunk, x1 - x0);
		*kname = xyz_name<BS, ZT, false, false>();
	}
}

template <int BS>
static bool launch_xyz_bs(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                          int x1, int xb0, int xb1, hipStream_t st, int ch, const FaceBC* fb,
                          const char** kn, const HetMaterials* het) {
	const int Z = g.sizes[2];
	if (Z <= 64) launch_xyz_t<BS, 64>(in, out, g, a, x0, x1, xb0, xb1, st, ch, fb, kn, het);
	else if (Z <= 128) launch_xyz_t<BS, 128>(in, out, g, a, x0, x1, xb0, xb1, st, ch, fb, kn, het);
	else if (Z <= 256) launch_xyz_t<BS, 256>(in, out, g, a, x0, x1, xb0, xb1, st, ch, fb, kn, het);
	else if (Z <= 512) launch_xyz_t<BS, 512>(in, out, g, a, x0, x1, xb0, xb1, st, ch, fb, kn, het);
	else launch_xyz_t<BS, 1024>(in, out, g, a, x0, x1, xb0, xb1, st, ch, fb, kn, het);
	return true;
}

#if GCMX_TX2_BLKT
// 8192 x 8 x 2 start / end times and 8192 HW_IDs of the last launch, then zeroed
#if GCMX_FMA
extern "C" int gcmx_diag_blk_fma(unsigned long long* t, unsigned* hw) {
#else
extern "C" int gcmx_diag_blk(unsigned long long* t, unsigned* hw) {
#endif
	if (hipDeviceSynchronize() != hipSuccess) return -1;
	if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_tx2_blk), sizeof(g_tx2_blk)) != hipSuccess) return -1;
	if (hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_tx2_hw), sizeof(g_tx2_hw)) != hipSuccess) return -1;
	static unsigned long long zero[kBlkMax][8][2];
	return hipMemcpyToSymbol(HIP_SYMBOL(g_tx2_blk), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

#if GCMX_TX2_DIAG && !GCMX_FMA
extern "C" int gcmx_diag_tx2(unsigned long long* out) {  // 16 x 8 counters, then reset
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tx2_diag), sizeof(g_tx2_diag)) != hipSuccess) return -1;
	static const unsigned long long zero[16][8] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_tx2_diag), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

bool launch_fused_xyz(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                      int x1, hipStream_t st, int chunk, const FaceBC* faces, const char** kname,
                      const HetMaterials* het, int xb0, int xb1) {
	const char* dummy = nullptr;
	const char** kn = kname ? kname : &dummy;
	if (!fused_supported(g) || x1 <= x0) return false;
	if (xb1 > xb0 && (xb0 < x1 || xb1 > g.sizes[0])) return false;  // range B after range A
	if (het && !het_supported(g)) return false;
	// the z split takes rows longer than 512 (and GCMX_ZS_PART's): uniform medium,
	// floor(q) = 0 -- then with face conditions and the folded ODE too
	const bool zs = !het && zs_admissible(g, a);
	if (faces && faces->on && !(fused_faces_supported(g) && (g.sizes[2] <= 512 || zs))) return false;
	if (faces && faces->ode_on && !(g.bs <= 2 && (g.sizes[2] <= 512 || zs))) return false;  // k_fused_xyz has no epilogue
	if (zs) {
		const int P = zs_part(g);
		const bool fc = faces && faces->on;
		auto go = [&](auto F) {
			constexpr bool FC = decltype(F)::value;
			if (g.bs == 1) P == 256 ? launch_zs<1, 256, FC>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn)
			               : launch_zs<1, 512, FC>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn);
			else P == 256 ? launch_zs<2, 256, FC>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn)
			              : launch_zs<2, 512, FC>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn);
		};
		if (fc) go(std::true_type{});
		else go(std::false_type{});
		return true;
	}
	switch (g.bs) {
	case 1: return launch_xyz_bs<1>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn, het);
	case 2: return launch_xyz_bs<2>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn, het);
	case 3: return launch_xyz_bs<3>(in, out, g, a, x0, x1, xb0, xb1, st, chunk, faces, kn, het);
	default: return false;
	}
}

}  // namespace GCMX_XYZ_NS

#if !GCMX_FMA
// CUs the one-pass step leaves free while it covers planes [x0, x1) in one
// round (the slab interior of the boundary-first schedule); 0 when its blocks
// fill every CU or it takes more than one round, -1 when k_step_tx2 does not run.
int step_free_cus(const Geo& g, int x0, int x1, int req_chunk, int cus_in) {
	const int Z = g.sizes[2];
	if (!fused_supported(g) || g.bs > 2 || Z > 512 || x1 <= x0) return -1;
	const int ZT = Z <= 64 ? 64 : Z <= 128 ? 128 : Z <= 256 ? 256 : 512;
	const int per_cu = 512 / ZT, cus = cus_in > 0 ? cus_in : GCMX_XYZ_NS::device_cus();
	const int npair = (x1 - x0 + ((g.gx0 + x0) & 1) + 1) / 2;
	const int chunk = GCMX_XYZ_NS::tx2_chunk_for(g.sizes[1], npair, req_chunk, cus * per_cu);
	const long long blocks = (long long)((g.sizes[1] + chunk - 1) / chunk) * npair;
	const long long slots = (long long)cus * per_cu;
	return blocks >= slots ? 0 : (int)((slots - blocks) / per_cu);
}

int zs_part(const Geo& g) {
	// GCMX_ZS_PART=256 (tuning): rows of 512 and more cut into 256-lane parts
	static const int env = [] {
		const char* e = std::getenv("GCMX_ZS_PART");
		return e ? std::atoi(e) : 0;
	}();
	const int Z = g.sizes[2];
	if (g.D != 3 || g.bs > 2) return 0;
	if (env == 256 && Z >= 512 && Z % 256 == 0) return 256;
	return Z > 512 && Z % 512 == 0 ? 512 : 0;
}


bool het_supported(const Geo& g) {
	const int Z = g.sizes[2];
	return fused_supported(g) && g.bs <= 2 && (Z == 64 || Z == 128 || Z == 256 || Z == 512);
}

bool fused_faces_supported(const Geo& g) {
	return fused_supported(g) && g.bs <= 2 && (g.sizes[2] <= 512 || zs_part(g) > 0) && g.sizes[1] >= 2 * g.bs + 2 &&
	       g.sizes[2] >= 2 * g.bs + 2;
}

bool zs_admissible(const Geo& g, const IsoAxis* a) {
	if (zs_part(g) <= 0) return false;
	for (int s = 0; s < 3; s++)
		if (a[s].kf1 != 0 || a[s].kf2 != 0) return false;
	return GCMX_XYZ_NS::same_axis(a[0], a[1]) && GCMX_XYZ_NS::same_axis(a[0], a[2]);
}

#endif

}  // namespace gcmx
