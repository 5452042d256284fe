// common.hpp -- device layout, per-axis stage tables and the Newton/min-max
// interpolation shared by every gcmx kernel.
//
// Layout: one time layer = M component planes (SoA).  A
// plane is the ghost-padded grid with the reference's axis order (X slowest,
// last axis fastest, CubicGrid.hpp:202-225).  The fastest axis is padded so
// that its first INNER node sits at a 128-byte boundary and every row is a
// multiple of 16 doubles: a wavefront reading 64 consecutive inner nodes of one
// component touches exactly four whole 128-byte lines.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcmx {

constexpr int kMaxM = 9;
constexpr int kMaxBs = 8;
constexpr int kRowAlign = 16;  // doubles (128 B)

__host__ __device__ constexpr int pde_size(int D) { return D + D * (D + 1) / 2; }

// Geometry of one context's device layers.
// Position of block b of a 1-D grid of T blocks in an XCD-contiguous order:
// blocks are dealt round-robin over the 8 XCDs (b % 8 share one,
// MI355X_MICROARCH.md §Workgroup dispatch), so XCD k, which receives
// ceil((T - k) / 8) blocks, gets the k-th contiguous run of positions.  Any T
// (a grid of 252 blocks used to fall back to the identity order and scatter
// neighbouring planes over the XCDs).
__device__ __forceinline__ int xcd_order(int b, int T) {
	const int q = T >> 3, r = T & 7, k = b & 7;
	return k * q + (k < r ? k : r) + (b >> 3);
}

struct Geo {
	int D, M, bs;
	int sizes[3];          // inner nodes (1 for axes >= D)
	long long stride[3];   // element strides (0 for axes >= D)
	long long origin;      // element offset of inner node (0,0,0)
	long long cs;          // component (plane) stride in elements
	long long n_inner;
	int lead;              // padding in front of the first ghost of a row
	long long row;         // padded length of the fastest axis
	int gx0;               // global x index of local plane 0 (CubicGrid::start[0])
};

// Per (material, axis) table: the matrices plus everything the stage derives
// from L and tau on the host (crossingPoints, GridCharacteristicMethod.hpp:56-59;
// q = |dx|/h and the Newton coefficients ((q - i) + 1) / i,
// EqualDistanceLineInterpolator.hpp:58-69), computed once per tau in IEEE double
// exactly as the reference does per node.
struct AxisTable {
	double U[kMaxM * kMaxM];
	double U1[kMaxM * kMaxM];
	double coef[kMaxM][kMaxBs];
	int shift[kMaxM];   // +1 / -1: side the characteristic foot lies on
	int kf[kMaxM];      // floor(q): interval holding the foot
	int zero_q[kMaxM];  // q == 0 exactly: interpolation returns the node value
	int pad_[kMaxM];
};

// v_max_f64 / v_min_f64 without the operand canonicalisation the compiler adds
// in front of fmax/fmin for values it cannot prove canonical (loads, LDS).
#ifndef GCMX_ASM_MINMAX
#define GCMX_ASM_MINMAX 1
#endif
#ifndef GCMX_CLAMP_MINMAX
#define GCMX_CLAMP_MINMAX 1
#endif
__device__ __forceinline__ double vmax(double a, double b) {
#if GCMX_ASM_MINMAX
	double r;
	asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
#else
	return fmax(a, b);
#endif
}
__device__ __forceinline__ double vmin(double a, double b) {
#if GCMX_ASM_MINMAX
	double r;
	asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
#else
	return fmin(a, b);
#endif
}

// The reference's limiter, `if (ans > max) ans = max; else if (ans < min) ans =
// min` with max / min of the segment ends a, b, returns the median of {ans, a, b}
// for every non-NaN input.  gfx950 has no v_med3_f64, and the clamp form
// min(max(ans, min(a, b)), max(a, b)) takes four v_*_f64; this one takes three:
//   lo = min(x, a), hi = max(x, a):  b >= hi -> hi;  b <= lo -> lo;  else b.
// Each result is one of the three inputs, so it is the clamp's value (only the
// sign of an exact zero may differ, as for the clamp form).
#ifndef GCMX_MED3
#define GCMX_MED3 1
#endif
__device__ __forceinline__ double vmed3(double x, double a, double b) {
	return vmax(vmin(x, a), vmin(vmax(x, a), b));
}
// limit(ans) for the segment (a, b)
__device__ __forceinline__ double vlimit(double ans, double a, double b) {
#if GCMX_MED3
	return vmed3(ans, a, b);
#else
	return vmin(vmax(ans, vmin(a, b)), vmax(a, b));
#endif
}

// EqualDistanceLineInterpolator::minMaxInterpolate for ONE component
// (EqualDistanceLineInterpolator.hpp:18-43 + 56-71).  s[0..BS] are the values
// at the node and its BS neighbours on the foot side.  The Newton recurrence
// is unrolled in the reference's order; the limiter bounds come from the
// original values s[kf], s[kf+1].
template <int BS, bool KF0 = false>
__device__ __forceinline__ double newton_minmax(const double (&s)[BS + 1], int kf,
                                                const double* __restrict__ coef) {
	// KF0: the caller knows floor(q) == 0 for every foot of the launch (Courant < 1)
	double lo = s[0], hi = s[1];
	if constexpr (!KF0) {
#pragma unroll
		for (int i = 1; i < BS; i++)
			if (kf == i) { lo = s[i]; hi = s[i + 1]; }
	}
	double d[BS + 1];
#pragma unroll
	for (int i = 0; i <= BS; i++) d[i] = s[i];
	double ans = d[0];
#pragma unroll
	for (int i = 1; i <= BS; i++) {
		const double c = coef[i - 1];
#pragma unroll
		for (int j = 0; j <= BS - i; j++) d[j] = (d[j + 1] - d[j]) * c;
		ans += d[0];
	}
	// if (ans > max) ans = max; else if (ans < min) ans = min;
	// == median(ans, lo, hi) for every non-NaN ans; only the sign of an exact zero
	// may differ.
#if GCMX_CLAMP_MINMAX
	return vlimit(ans, lo, hi);
#else
	const double mx = vmax(lo, hi), mn = vmin(lo, hi);
	return (ans > mx) ? mx : ((ans < mn) ? mn : ans);
#endif
}

// Same with compile-time coefficients held in registers by the caller.
template <int BS>
__device__ __forceinline__ double newton_minmax_r(const double (&s)[BS + 1], int kf,
                                                  const double (&coef)[BS]) {
	return newton_minmax<BS>(s, kf, coef);
}

}  // namespace gcmx
