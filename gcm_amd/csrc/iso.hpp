// iso.hpp -- device-side structure of the isotropic-elastic stage shared by the
// fast kernels (kernels_fast.hip: march / line / fused Y-Z; kernels_xyz.hip: the
// one-pass X/Y/Z step).  See kernels_fast.hip for the derivation.
#pragma once

#include "common.hpp"
#include "launch.hpp"

namespace gcmx {

// ----------------------------------------------------------- structure --

// Index of sigma(i,j) in the 3-D PDE vector (VelocitySigmaVariables.hpp:82-96).
__host__ __device__ constexpr int sig3(int i, int j) {
	return (i <= j) ? 3 + (i * 3 - ((i - 1) * i) / 2 + j - i)
	                : 3 + (j * 3 - ((j - 1) * j) / 2 + i - j);
}
__host__ __device__ constexpr unsigned bit(int i) { return 1u << i; }

// createLocalBasis(e_s) (linal/basis.hpp:58-65, geometry.hpp:35-52): the two
// tangents are +-e_t1, +-e_t2 with these axes and signs.
__host__ __device__ constexpr int tang1(int s) { return s == 0 ? 1 : 0; }
__host__ __device__ constexpr int tang2(int s) { return s == 2 ? 1 : 2; }
__host__ __device__ constexpr int sgn1(int s) { return s == 0 ? -1 : 1; }
__host__ __device__ constexpr int sgn2(int s) { return s == 2 ? 1 : -1; }

// A matrix entry: `sign * (slot value or constant)`.
enum Slot : int { kZero = 0, kOne, kHalf, kA, kB, kG, kP1, kP2, kS };
struct Coef {
	int slot;
	int sign;
};
__host__ __device__ constexpr Coef cz() { return Coef{kZero, 0}; }

// U(k, j) (ElasticModel.hpp:486-553): rows are eigenstrings.
__host__ __device__ constexpr Coef iso_u(int S, int k, int j) {
	const int t1 = tang1(S), t2 = tang2(S), s1 = sgn1(S), s2 = sgn2(S);
	const int ss = sig3(S, S), st1 = sig3(t1, S), st2 = sig3(t2, S);
	const int s11 = sig3(t1, t1), s22 = sig3(t2, t2), s12 = sig3(t1, t2);
	return (k == 0) ? (j == S ? Coef{kOne, 1} : j == ss ? Coef{kA, 1} : cz())
	     : (k == 1) ? (j == S ? Coef{kOne, 1} : j == ss ? Coef{kA, -1} : cz())
	     : (k == 2) ? (j == t1 ? Coef{kOne, s1} : j == st1 ? Coef{kB, s1} : cz())
	     : (k == 3) ? (j == t1 ? Coef{kOne, s1} : j == st1 ? Coef{kB, -s1} : cz())
	     : (k == 4) ? (j == t2 ? Coef{kOne, s2} : j == st2 ? Coef{kB, s2} : cz())
	     : (k == 5) ? (j == t2 ? Coef{kOne, s2} : j == st2 ? Coef{kB, -s2} : cz())
	     : (k == 6) ? (j == s12 ? Coef{kOne, s1 * s2} : cz())
	     : (k == 7) ? (j == s11 ? Coef{kOne, 1} : j == s22 ? Coef{kOne, -1} : cz())
	                : (j == s11 ? Coef{kOne, 1} : j == s22 ? Coef{kOne, 1}
	                   : j == ss ? Coef{kG, 1} : cz());
}

// U1(c, n) (ElasticModel.hpp:416-483): columns are eigenvectors.
__host__ __device__ constexpr Coef iso_u1(int S, int c, int n) {
	const int t1 = tang1(S), t2 = tang2(S), s1 = sgn1(S), s2 = sgn2(S);
	const int ss = sig3(S, S), st1 = sig3(t1, S), st2 = sig3(t2, S);
	const int s11 = sig3(t1, t1), s22 = sig3(t2, t2), s12 = sig3(t1, t2);
	return (n == 0) ? (c == S ? Coef{kHalf, 1} : c == ss ? Coef{kP1, 1}
	                   : (c == s11 || c == s22) ? Coef{kP2, 1} : cz())
	     : (n == 1) ? (c == S ? Coef{kHalf, 1} : c == ss ? Coef{kP1, -1}
	                   : (c == s11 || c == s22) ? Coef{kP2, -1} : cz())
	     : (n == 2) ? (c == t1 ? Coef{kHalf, s1} : c == st1 ? Coef{kS, s1} : cz())
	     : (n == 3) ? (c == t1 ? Coef{kHalf, s1} : c == st1 ? Coef{kS, -s1} : cz())
	     : (n == 4) ? (c == t2 ? Coef{kHalf, s2} : c == st2 ? Coef{kS, s2} : cz())
	     : (n == 5) ? (c == t2 ? Coef{kHalf, s2} : c == st2 ? Coef{kS, -s2} : cz())
	     : (n == 6) ? (c == s12 ? Coef{kOne, s1 * s2} : cz())
	     : (n == 7) ? (c == s11 ? Coef{kHalf, 1} : c == s22 ? Coef{kHalf, -1} : cz())
	                : (c == s11 ? Coef{kHalf, 1} : c == s22 ? Coef{kHalf, 1} : cz());
}

// Components read at the neighbours (rows 0..5) / only at the node (rows 6..8).
__host__ __device__ constexpr unsigned iso_window(int S) {
	unsigned m = 0;
	for (int k = 0; k < 6; k++)
		for (int j = 0; j < 9; j++)
			if (iso_u(S, k, j).slot != kZero) m |= bit(j);
	return m;
}
__host__ __device__ constexpr unsigned iso_center_only(int S) {
	unsigned m = 0;
	for (int k = 6; k < 9; k++)
		for (int j = 0; j < 9; j++)
			if (iso_u(S, k, j).slot != kZero) m |= bit(j);
	return m & ~iso_window(S);
}
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
// u * v for a structural entry; exact w.r.t. the reference product fl(u * v).
template <int SLOT, int SIGN>
__device__ __forceinline__ double term(const IsoAxis& A, double v) {
	double m;
	if constexpr (SLOT == kOne) m = v;
	else if constexpr (SLOT == kHalf) m = v * 0.5;
	else if constexpr (SLOT == kA) m = A.a * v;
	else if constexpr (SLOT == kB) m = A.b * v;
	else if constexpr (SLOT == kG) m = A.g * v;
	else if constexpr (SLOT == kP1) m = A.p1 * v;
	else if constexpr (SLOT == kP2) m = A.p2 * v;
	else m = A.s * v;
	return SIGN > 0 ? m : -m;
}

// Unrolled sum over j of U(k, j) * V(j) (or U1(c, n) * r(n)) in ascending index
// order, skipping structural zeros, starting from the first non-zero term.
template <int S, bool ISU1, int ROW, int J = 0>
struct RowSum {
	template <class F>
	__device__ __forceinline__ static double go(const IsoAxis& A, F val, double acc, bool first) {
		if constexpr (J == 9) {
			return acc;
		} else {
			constexpr Coef c = ISU1 ? iso_u1(S, ROW, J) : iso_u(S, ROW, J);
			if constexpr (c.slot == kZero) {
				return RowSum<S, ISU1, ROW, J + 1>::go(A, val, acc, first);
			} else {
				const double t = term<c.slot, c.sign>(A, val(J));
				return RowSum<S, ISU1, ROW, J + 1>::go(A, val, first ? t : acc + t, false);
			}
		}
	}
};

// Components of characteristic pair P (rows 2P, 2P+1 of U): the velocity
// component and the stress component each row reads at the feet.
__host__ __device__ constexpr int pair_vel(int S, int P) { return P == 0 ? S : P == 1 ? tang1(S) : tang2(S); }
__host__ __device__ constexpr int pair_sig(int S, int P) {
	return P == 0 ? sig3(S, S) : P == 1 ? sig3(tang1(S), S) : sig3(tang2(S), S);
}

// GCMX_LAGRANGE (the one-pass step's FMA build, kernels_xyz.hip compiled with
// GCMX_FMA=1): with floor(q) = 0 and bs <= 2 a foot's interpolant is evaluated
// in Lagrange form, w0 s0 + w1 s1 + w2 s2 with the host's weights
// (lagrange_weights), as one multiply and bs fused multiply-adds: the same
// polynomial as minMaxInterpolate's Newton form (EqualDistanceLineInterpolator.hpp:56-71)
// with other roundings, ~1e-16 relative, inside the north star's 1e-10 of the
// reference; the min-max limiter is unchanged.  The exact build
// keeps the reference's Newton operations.
#ifndef GCMX_FMA
#define GCMX_FMA 0
#endif
#ifndef GCMX_LAGRANGE
#define GCMX_LAGRANGE GCMX_FMA
#endif
template <int BS>
__device__ __forceinline__ double lagrange_minmax(const double (&s)[BS + 1], const double* __restrict__ w) {
	double ans = s[0] * w[0];
#pragma unroll
	for (int i = 1; i <= BS; i++) ans = __builtin_fma(w[i], s[i], ans);
	return vlimit(ans, s[0], s[1]);
}

// Rows 2P (foot on the -S side, L > 0) and 2P+1 (+S side) of r = diag(U * V):
// the two interpolations per component (minMaxInterpolate) and the U row sums.
// W(j, o): component j at offset o along S (|o| <= BS).
template <int S, int BS, bool KF0, int P, class WF>
__device__ __forceinline__ void pair_update(const IsoAxis& A, WF W, double& ra, double& rb) {
	const double* coef = (P == 0) ? A.c1 : A.c2;
	const double* wts = (P == 0) ? A.w1 : A.w2;
	const int kf = (P == 0) ? A.kf1 : A.kf2;
	auto interp = [&](int j, int sh) {
		double sv[BS + 1];
#pragma unroll
		for (int i = 0; i <= BS; i++) sv[i] = W(j, sh * i);
		if constexpr (GCMX_LAGRANGE && KF0 && BS <= 2) return lagrange_minmax<BS>(sv, wts);
		else return newton_minmax<BS, KF0>(sv, kf, coef);
	};
	ra = RowSum<S, false, 2 * P>::go(A, [&](int j) { return interp(j, -1); }, 0.0, true);
	rb = RowSum<S, false, 2 * P + 1>::go(A, [&](int j) { return interp(j, 1); }, 0.0, true);
}

// Rows 6..8 (q == 0: the interpolant is the node value itself).  C(j): node value.
template <int S, class CF>
__device__ __forceinline__ void center_update(const IsoAxis& A, CF C, double (&r)[9]) {
	r[6] = RowSum<S, false, 6>::go(A, C, 0.0, true);
	r[7] = RowSum<S, false, 7>::go(A, C, 0.0, true);
	r[8] = RowSum<S, false, 8>::go(A, C, 0.0, true);
}

// out = U1 * r (localGcmStep's second product).
template <int S>
__device__ __forceinline__ void u1_apply(const IsoAxis& A, const double (&r)[9], double (&out)[9]) {
	auto rv = [&](int n) { return r[n]; };
	out[0] = RowSum<S, true, 0>::go(A, rv, 0.0, true);
	out[1] = RowSum<S, true, 1>::go(A, rv, 0.0, true);
	out[2] = RowSum<S, true, 2>::go(A, rv, 0.0, true);
	out[3] = RowSum<S, true, 3>::go(A, rv, 0.0, true);
	out[4] = RowSum<S, true, 4>::go(A, rv, 0.0, true);
	out[5] = RowSum<S, true, 5>::go(A, rv, 0.0, true);
	out[6] = RowSum<S, true, 6>::go(A, rv, 0.0, true);
	out[7] = RowSum<S, true, 7>::go(A, rv, 0.0, true);
	out[8] = RowSum<S, true, 8>::go(A, rv, 0.0, true);
}

// One node's stage.  W(j, o): window component j at offset o along S
// (|o| <= BS); C(j): node value of a component rows 6..8 read.
template <int S, int BS, bool KF0, class WF, class CF>
__device__ __forceinline__ void node_update(const IsoAxis& A, WF W, CF C, double (&out)[9]) {
	double r[9];
	pair_update<S, BS, KF0, 0>(A, W, r[0], r[1]);
	pair_update<S, BS, KF0, 1>(A, W, r[2], r[3]);
	pair_update<S, BS, KF0, 2>(A, W, r[4], r[5]);
	center_update<S>(A, C, r);
	u1_apply<S>(A, r, out);
}

// Per-component plane base pointers are uniform; per-thread offsets are 32-bit
// element indices (layer planes are < 2^29 elements, checked on the host).  The
// nine bases are made opaque SGPR values once per kernel so that every access
// is the scalar-base + 32-bit-VGPR-offset form (one shared offset register, no
// 64-bit address arithmetic per component).
typedef const __attribute__((address_space(1))) double* gcptr;
typedef __attribute__((address_space(1))) double* gptr;
#ifndef GCMX_SGPR_BASES
#define GCMX_SGPR_BASES 1
#endif
__device__ __forceinline__ gcptr sgpr_ptr(const double* p) {
	gcptr q = (gcptr)p;
#if GCMX_SGPR_BASES
	asm volatile("" : "+s"(q));
#endif
	return q;
}
__device__ __forceinline__ gptr sgpr_ptr(double* p) {
	gptr q = (gptr)p;
#if GCMX_SGPR_BASES
	asm volatile("" : "+s"(q));
#endif
	return q;
}
struct Planes {
	gcptr b[kMaxM];
	__device__ __forceinline__ Planes(const double* p, long long cs) {
#pragma unroll
		for (int j = 0; j < kMaxM; j++) b[j] = sgpr_ptr(p + j * cs);
	}
	__device__ __forceinline__ double ld(int j, unsigned off) const {
		typedef const __attribute__((address_space(1))) char* gcb;
		return *reinterpret_cast<gcptr>(reinterpret_cast<gcb>(b[j]) + (size_t)(off << 3));
	}
};
struct PlanesW {
	gptr b[kMaxM];
	__device__ __forceinline__ PlanesW(double* p, long long cs) {
#pragma unroll
		for (int j = 0; j < kMaxM; j++) b[j] = sgpr_ptr(p + j * cs);
	}
	__device__ __forceinline__ void st(int j, unsigned off, double v) const {
		typedef __attribute__((address_space(1))) char* gb;
		*reinterpret_cast<gptr>(reinterpret_cast<gb>(b[j]) + (size_t)(off << 3)) = v;
	}
	__device__ __forceinline__ void st_nt(int j, unsigned off, double v) const {
		typedef __attribute__((address_space(1))) char* gb;
		__builtin_nontemporal_store(v, reinterpret_cast<gptr>(reinterpret_cast<gb>(b[j]) + (size_t)(off << 3)));
	}
};

// Byte-offset form: the 32-bit per-lane offset is made opaque, so every access
// is `global_load_dwordx2 v, v_off, s[base]` (SGPR base + 32-bit VGPR offset,
// the global "saddr" form) and the components that share an offset share its
// VGPR; otherwise hipcc tends to materialise 64-bit addresses
// (v_lshl_add_u64 per load).  `boff` = element offset * 8 (< 2^32: planes are
// < 2^32 bytes, fast_layout_ok).  The asm is not volatile, so equal offsets CSE.
__device__ __forceinline__ unsigned opaque_u32(unsigned x) {
	asm("" : "+v"(x));
	return x;
}
__device__ __forceinline__ double ld_b(const Planes& p, int j, unsigned boff) {
	typedef const __attribute__((address_space(1))) char* gcb;
	return *reinterpret_cast<gcptr>(reinterpret_cast<gcb>(p.b[j]) + (unsigned long long)boff);
}
// single-use load (streaming: no L2 allocation preference over the reused planes)
__device__ __forceinline__ double ld_nt_b(const Planes& p, int j, unsigned boff) {
	typedef const __attribute__((address_space(1))) char* gcb;
	return __builtin_nontemporal_load(reinterpret_cast<gcptr>(reinterpret_cast<gcb>(p.b[j]) + (unsigned long long)boff));
}
__device__ __forceinline__ void st_b(const PlanesW& p, int j, unsigned boff, double v) {
	typedef __attribute__((address_space(1))) char* gb;
	*reinterpret_cast<gptr>(reinterpret_cast<gb>(p.b[j]) + (unsigned long long)boff) = v;
}
__device__ __forceinline__ void st_nt_b(const PlanesW& p, int j, unsigned boff, double v) {
	typedef __attribute__((address_space(1))) char* gb;
	__builtin_nontemporal_store(v, reinterpret_cast<gptr>(reinterpret_cast<gb>(p.b[j]) + (unsigned long long)boff));
}

}  // namespace gcmx
