// contact.hpp -- per-node arithmetic of the simplex contact correctors
// (engine/simplex/ContactCorrector.hpp, engine/simplex/common.hpp:170-260,
// rheology/models/ElasticModel.hpp:157-300), shared by the device kernels
// (simplex.hip) and the host set-up (gcm_amd/host/simplex.cpp: the
// getMaximalPossibleDeterminants thresholds).  Every expression keeps the
// reference's evaluation order; compiled with -ffp-contract=off on both sides.
//
// PDE vector order: Vx Vy Vz Sxx Sxy Sxz Syy Syz Szz (VelocitySigmaVariables.hpp:82-96).
#pragma once

#include <cmath>

#ifdef __HIPCC__
#define GSX_HD __host__ __device__ inline
#else
#define GSX_HD inline
#endif

namespace gsx {

constexpr int M = 9;

/// Symmetric-storage slot of sigma(i, j) (linal/Symmetry.hpp:38-46).
GSX_HD int sym(int i, int j) {
	const int a = i < j ? i : j, b = i < j ? j : i;
	return 3 + a * 3 - ((a - 1) * a) / 2 + b - a;
}

/// linal::determinant of 3x3 (determinants.hpp:40-53).
GSX_HD double det3(double m11, double m12, double m13, double m21, double m22, double m23,
                   double m31, double m32, double m33) {
	return m11 * (m22 * m33 - m23 * m32) - m12 * (m21 * m33 - m23 * m31) +
	       m13 * (m21 * m32 - m22 * m31);
}
GSX_HD double det3(const double (&A)[3][3]) {
	return det3(A[0][0], A[0][1], A[0][2], A[1][0], A[1][1], A[1][2], A[2][0], A[2][1], A[2][2]);
}

/// linal::solveLinearSystem 3x3 by Cramer (linearSystems.hpp:104-129); the caller
/// guarantees det != 0.
GSX_HD void solve3(const double (&A)[3][3], const double (&b)[3], double (&x)[3]) {
	const double det = det3(A);
	const double d1 = det3(b[0], A[0][1], A[0][2], b[1], A[1][1], A[1][2], b[2], A[2][1], A[2][2]);
	const double d2 = det3(A[0][0], b[0], A[0][2], A[1][0], b[1], A[1][2], A[2][0], b[2], A[2][2]);
	const double d3 = det3(A[0][0], A[0][1], b[0], A[1][0], A[1][1], b[1], A[2][0], A[2][1], b[2]);
	x[0] = d1 / det;
	x[1] = d2 / det;
	x[2] = d3 / det;
}

/// linal::invert 3x3 (functions.hpp:128-134): cofactors / determinant.
GSX_HD void invert3(const double (&m)[3][3], double (&r)[3][3]) {
	const double c[9] = {m[1][1] * m[2][2] - m[1][2] * m[2][1], m[0][2] * m[2][1] - m[0][1] * m[2][2],
	                     m[0][1] * m[1][2] - m[1][1] * m[0][2], m[1][2] * m[2][0] - m[1][0] * m[2][2],
	                     m[0][0] * m[2][2] - m[0][2] * m[2][0], m[0][2] * m[1][0] - m[0][0] * m[1][2],
	                     m[1][0] * m[2][1] - m[1][1] * m[2][0], m[0][1] * m[2][0] - m[0][0] * m[2][1],
	                     m[0][0] * m[1][1] - m[0][1] * m[1][0]};
	const double det = det3(m);
	for (int i = 0; i < 9; i++) r[i / 3][i % 3] = c[i] / det;
}

/// ElasticModel::borderMatrixFixedVelocityGlobalBasis (ElasticModel.hpp:183-194): B1.
GSX_HD void fixedVelocityGlobal(double (&B)[3][M]) {
	for (int i = 0; i < 3; i++)
		for (int k = 0; k < M; k++) B[i][k] = (k == i) ? 1.0 : 0.0;
}
/// ElasticModel::borderMatrixFixedForceGlobalBasis (ElasticModel.hpp:162-176): B2,
/// row i: sigma(i, j) = n(j) in symmetric storage (the later j overwrites).
GSX_HD void fixedForceGlobal(const double (&n)[3], double (&B)[3][M]) {
	for (int i = 0; i < 3; i++) {
		for (int k = 0; k < M; k++) B[i][k] = 0.0;
		for (int j = 0; j < 3; j++) B[i][sym(i, j)] = n[j];
	}
}

/// (3 x 9) * (9 x 3) with Omega = U1's columns `cols` (getColumnsFromGcmMatrices,
/// common.hpp:153-165); operator* order (operators.hpp:109-123).
GSX_HD void mulBOmega(const double (&B)[3][M], const double* U1, const int (&cols)[3],
                      double (&R)[3][3]) {
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) {
			double x = B[i][0] * U1[0 * M + cols[j]];
			for (int n = 1; n < M; n++) x += B[i][n] * U1[n * M + cols[j]];
			R[i][j] = x;
		}
}
GSX_HD void mulBu(const double (&B)[3][M], const double (&u)[M], double (&r)[3]) {
	for (int i = 0; i < 3; i++) {
		double x = B[i][0] * u[0];
		for (int n = 1; n < M; n++) x += B[i][n] * u[n];
		r[i] = x;
	}
}
GSX_HD void mul33(const double (&A)[3][3], const double (&B)[3][3], double (&C)[3][3]) {
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) {
			double x = A[i][0] * B[0][j];
			x += A[i][1] * B[1][j];
			x += A[i][2] * B[2][j];
			C[i][j] = x;
		}
}
GSX_HD void mul33v(const double (&A)[3][3], const double (&v)[3], double (&r)[3]) {
	for (int i = 0; i < 3; i++) {
		double x = A[i][0] * v[0];
		x += A[i][1] * v[1];
		x += A[i][2] * v[2];
		r[i] = x;
	}
}
/// Omega * alpha (9 x 3 times 3).
GSX_HD void mulOmega(const double* U1, const int (&cols)[3], const double (&a)[3],
                     double (&v)[M]) {
	for (int i = 0; i < M; i++) {
		double x = U1[i * M + cols[0]] * a[0];
		x += U1[i * M + cols[1]] * a[1];
		x += U1[i * M + cols[2]] * a[2];
		v[i] = x;
	}
}

struct ContactCorrection {
	double det1 = 0, det2 = 0;
	bool ok = false;
	double valueA[M], valueB[M];
};

/// The two-body calculateOuterWaveCorrection (common.hpp:220-260) for
/// B1A = B1B = FixedVelocityGlobalBasis and B2A = B2B = FixedForceGlobalBasis(n)
/// (AdhesionContactMatrixCreator, ContactCorrector.hpp:466-483; both models elastic).
GSX_HD ContactCorrection contactCorrection(const double (&uA)[M], const double* U1A,
                                           const int (&colsA)[3], const double (&uB)[M],
                                           const double* U1B, const int (&colsB)[3],
                                           const double (&B1)[3][M], const double (&B2)[3][M],
                                           double minValid1, double minValid2) {
	ContactCorrection ans;
	for (int k = 0; k < M; k++) ans.valueA[k] = ans.valueB[k] = 0.0;
	double R1[3][3];
	mulBOmega(B1, U1A, colsA, R1);  // R1 = B1A * OmegaA
	ans.det1 = std::fabs(det3(R1));
	ans.ok = ans.det1 > minValid1;
	if (!ans.ok) return ans;
	double R[3][3];
	invert3(R1, R);
	double b1B[3], b1A[3], d[3], p[3];
	mulBu(B1, uB, b1B);
	mulBu(B1, uA, b1A);
	for (int i = 0; i < 3; i++) d[i] = b1B[i] - b1A[i];
	mul33v(R, d, p);  // p = R * (B1B * uB - B1A * uA)
	double B1OB[3][3], Q[3][3];
	mulBOmega(B1, U1B, colsB, B1OB);
	mul33(R, B1OB, Q);  // Q = R * (B1B * OmegaB)
	double B2OB[3][3], B2OA[3][3], B2OAQ[3][3], A[3][3];
	mulBOmega(B2, U1B, colsB, B2OB);
	mulBOmega(B2, U1A, colsA, B2OA);
	mul33(B2OA, Q, B2OAQ);
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) A[i][j] = B2OB[i][j] - B2OAQ[i][j];
	double t[3], b2A[3], b2B[3], f[3];
	mul33v(B2OA, p, t);
	mulBu(B2, uA, b2A);
	mulBu(B2, uB, b2B);
	for (int i = 0; i < 3; i++) f[i] = (t[i] + b2A[i]) - b2B[i];
	ans.det2 = std::fabs(det3(A));
	ans.ok = ans.det2 > minValid2;
	if (!ans.ok) return ans;
	double alphaB[3], Qa[3], alphaA[3];
	solve3(A, f, alphaB);
	mul33v(Q, alphaB, Qa);
	for (int i = 0; i < 3; i++) alphaA[i] = p[i] + Qa[i];
	mulOmega(U1A, colsA, alphaA, ans.valueA);
	mulOmega(U1B, colsB, alphaB, ans.valueB);
	return ans;
}

// ---- GSL restatement for the 6 x 6 systems (util/math/GslUtils.hpp:96-168) ----
// gsl_linalg_LU_decomp (GSL lu.c: Doolittle, partial pivoting on the first
// strictly largest |a_ij|), gsl_linalg_LU_det, gsl_linalg_LU_solve (permute,
// then the unit-lower and upper cblas dtrsv sweeps).  GSL is not in this image
// and not vendored by the reference; this is the classic (pre-2.6) algorithm.
constexpr int N6 = 6;

template <int N>
GSX_HD void luDecomp(double (&A)[N][N], int (&perm)[N], int& signum) {
	signum = 1;
	for (int i = 0; i < N; i++) perm[i] = i;
	for (int j = 0; j < N - 1; j++) {
		double mx = std::fabs(A[j][j]);
		int piv = j;
		for (int i = j + 1; i < N; i++) {
			const double aij = std::fabs(A[i][j]);
			if (aij > mx) {
				mx = aij;
				piv = i;
			}
		}
		if (piv != j) {
			for (int k = 0; k < N; k++) {
				const double t = A[j][k];
				A[j][k] = A[piv][k];
				A[piv][k] = t;
			}
			const int t = perm[j];
			perm[j] = perm[piv];
			perm[piv] = t;
			signum = -signum;
		}
		const double ajj = A[j][j];
		if (ajj != 0.0) {
			for (int i = j + 1; i < N; i++) {
				const double aij = A[i][j] / ajj;
				A[i][j] = aij;
				for (int k = j + 1; k < N; k++) A[i][k] = A[i][k] - aij * A[j][k];
			}
		}
	}
}
template <int N>
GSX_HD double luDet(const double (&LU)[N][N], int signum) {
	double det = (double)signum;
	for (int i = 0; i < N; i++) det *= LU[i][i];
	return det;
}
// gsl_linalg_LU_solve refuses a singular factorisation (a zero on U's
// diagonal: "matrix is singular", GSL_EDOM); the callers check it first.
template <int N>
GSX_HD bool luSingular(const double (&LU)[N][N]) {
	for (int i = 0; i < N; i++)
		if (LU[i][i] == 0.0) return true;
	return false;
}
template <int N>
GSX_HD void luSolve(const double (&LU)[N][N], const int (&perm)[N], const double (&b)[N], double (&x)[N]) {
	for (int i = 0; i < N; i++) x[i] = b[perm[i]];  // gsl_permute_vector: x'_i = x_{p_i}
	for (int i = 1; i < N; i++) {                // L, unit diagonal
		double t = x[i];
		for (int j = 0; j < i; j++) t -= LU[i][j] * x[j];
		x[i] = t;
	}
	x[N - 1] = x[N - 1] / LU[N - 1][N - 1];  // U
	for (int i = N - 2; i >= 0; i--) {
		double t = x[i];
		for (int j = i + 1; j < N; j++) t -= LU[i][j] * x[j];
		x[i] = t / LU[i][i];
	}
}
GSX_HD void luDecomp6(double (&A)[N6][N6], int (&perm)[N6], int& signum) { luDecomp<N6>(A, perm, signum); }
GSX_HD double luDet6(const double (&LU)[N6][N6], int signum) { return luDet<N6>(LU, signum); }
GSX_HD void luSolve6(const double (&LU)[N6][N6], const int (&perm)[N6], const double (&b)[N6], double (&x)[N6]) {
	luSolve<N6>(LU, perm, b, x);
}

/// The contact node that is a border with two conditions (ContactCorrector.hpp:
/// 176-218): B = [B1; B2] (6 x 9), Omega = [RIGHT | LEFT] columns of U1 (9 x 6),
/// b12 = [B1 * uOther; B2 * uOther]; the one-body calculateOuterWaveCorrection
/// (common.hpp:179-197) with the 6 x 6 determinant / solve through GSL.
GSX_HD bool doubleBorderCorrection(const double (&u)[M], const double* U1,
                                   const double (&uOther)[M], const double (&B1)[3][M],
                                   const double (&B2)[3][M], double minValid, double (&value)[M]) {
	const int cols[6] = {1, 3, 5, 0, 2, 4};  // RIGHT_INVARIANTS, LEFT_INVARIANTS (Model.cpp:81-82)
	double Bm[N6][M];
	for (int i = 0; i < 3; i++)
		for (int k = 0; k < M; k++) {
			Bm[i][k] = B1[i][k];
			Bm[i + 3][k] = B2[i][k];
		}
	double Mm[N6][N6];
	for (int i = 0; i < N6; i++)
		for (int j = 0; j < N6; j++) {
			double x = Bm[i][0] * U1[0 * M + cols[j]];
			for (int n = 1; n < M; n++) x += Bm[i][n] * U1[n * M + cols[j]];
			Mm[i][j] = x;
		}
	double LU[N6][N6];
	for (int i = 0; i < N6; i++)
		for (int j = 0; j < N6; j++) LU[i][j] = Mm[i][j];
	int perm[N6], signum;
	luDecomp6(LU, perm, signum);
	const double detFabs = std::fabs(luDet6(LU, signum));
	if (!(detFabs > minValid)) return false;
	double rhs[N6];
	for (int i = 0; i < N6; i++) {
		double b12 = Bm[i][0] * uOther[0];  // b12 = concat(B1 * uOther, B2 * uOther)
		for (int n = 1; n < M; n++) b12 += Bm[i][n] * uOther[n];
		double Bu = Bm[i][0] * u[0];
		for (int n = 1; n < M; n++) Bu += Bm[i][n] * u[n];
		rhs[i] = b12 - Bu;
	}
	double alpha[N6];
	luSolve6(LU, perm, rhs, alpha);  // solveLinearSystem re-decomposes the same matrix
	for (int i = 0; i < M; i++) {
		double x = U1[i * M + cols[0]] * alpha[0];
		for (int j = 1; j < N6; j++) x += U1[i * M + cols[j]] * alpha[j];
		value[i] = x;
	}
	return true;
}

// ---- plain contact corrections (ElasticModel.hpp:230-300), S = createLocalBasis(n) ----
GSX_HD void sigmaToLocal(const double (&u)[M], const double (&S)[3][3], double (&sl)[3][3]) {
	double sg[3][3], t[3][3];
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) sg[i][j] = u[sym(i, j)];  // getSigmaFrom
	for (int i = 0; i < 3; i++)                              // S_T * sigmaGlobal
		for (int j = 0; j < 3; j++) {
			double x = S[0][i] * sg[0][j];
			x += S[1][i] * sg[1][j];
			x += S[2][i] * sg[2][j];
			t[i][j] = x;
		}
	for (int i = 0; i < 3; i++)  // (...) * S
		for (int j = 0; j < 3; j++) {
			double x = t[i][0] * S[0][j];
			x += t[i][1] * S[1][j];
			x += t[i][2] * S[2][j];
			sl[i][j] = x;
		}
}
GSX_HD void sigmaFromLocal(double (&u)[M], const double (&S)[3][3], const double (&sl)[3][3]) {
	double t[3][3];
	for (int i = 0; i < 3; i++)  // S * sigmaLocal
		for (int j = 0; j < 3; j++) {
			double x = S[i][0] * sl[0][j];
			x += S[i][1] * sl[1][j];
			x += S[i][2] * sl[2][j];
			t[i][j] = x;
		}
	for (int i = 0; i < 3; i++)  // (...) * S_T, then setSigmaTo (row-major writes)
		for (int j = 0; j < 3; j++) {
			double x = t[i][0] * S[j][0];
			x += t[i][1] * S[j][1];
			x += t[i][2] * S[j][2];
			u[sym(i, j)] = x;
		}
}
/// applyPlainContactCorrectionAsAverage (ElasticModel.hpp:239-272), ADHESION.
GSX_HD void plainContactAverage(double (&uA)[M], double (&uB)[M], const double (&S)[3][3]) {
	for (int i = 0; i < 3; i++) {
		const double v = (uA[i] + uB[i]) / 2;
		uA[i] = v;
		uB[i] = v;
	}
	double lA[3][3], lB[3][3], sn[3];
	sigmaToLocal(uA, S, lA);
	sigmaToLocal(uB, S, lB);
	for (int i = 0; i < 3; i++) sn[i] = (lA[i][2] + lB[i][2]) / 2;
	for (int i = 0; i < 3; i++) {
		lA[i][2] = sn[i];
		lB[i][2] = sn[i];
	}
	for (int j = 0; j < 3; j++) {
		lA[2][j] = sn[j];
		lB[2][j] = sn[j];
	}
	sigmaFromLocal(uA, S, lA);
	sigmaFromLocal(uB, S, lB);
}
/// applyPlainContactCorrection (ElasticModel.hpp:279-300): uA takes uB's velocity
/// and normal traction.
GSX_HD void plainContactOneSided(double (&uA)[M], const double (&uB)[M], const double (&S)[3][3]) {
	for (int i = 0; i < 3; i++) uA[i] = uB[i];
	double lA[3][3], lB[3][3], sn[3];
	sigmaToLocal(uA, S, lA);
	sigmaToLocal(uB, S, lB);
	for (int i = 0; i < 3; i++) sn[i] = lB[i][2];
	for (int i = 0; i < 3; i++) lA[i][2] = sn[i];
	for (int j = 0; j < 3; j++) lA[2][j] = sn[j];
	sigmaFromLocal(uA, S, lA);
}

}  // namespace gsx
