/*
 * gcm_oracle.c -- CPU restatement of the reference cubic GCM stage path.
 * TEST INFRASTRUCTURE ONLY (see gcm_oracle.h).  Every function follows the
 * reference operation by operation, in the same floating-point order, so that
 * its results are bitwise those of libgcm compiled for x86-64 without FMA.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "gcm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OG_MAXM 9
#define OG_MAXBS 16

/* ---------------------------------------------------------------- grid -- */

/* CubicGrid.hpp:202-225 (calculateIndexMaker): X slowest, last axis fastest. */
void og_index_maker(const og_grid* g, long long im[3]) {
	const long long b2 = 2LL * g->bs;
	im[0] = im[1] = im[2] = 0;
	switch (g->D) {
	case 1: im[0] = 1; break;
	case 2: im[0] = b2 + g->sizes[1]; im[1] = 1; break;
	case 3:
		im[0] = (b2 + g->sizes[1]) * (b2 + g->sizes[2]);
		im[1] = b2 + g->sizes[2];
		im[2] = 1;
		break;
	}
}

/* CubicGrid.hpp:132-134 */
long long og_size_of_all_nodes(const og_grid* g) {
	long long im[3];
	og_index_maker(g, im);
	return im[0] * (2LL * g->bs + g->sizes[0]);
}

/* CubicGrid.hpp:141-147 */
static long long og_get_index(const og_grid* g, const long long im[3], const int it[3]) {
	long long ans = 0;
	for (int i = 0; i < g->D; i++) ans += im[i] * (long long)(it[i] + g->bs);
	return ans;
}

/* ------------------------------------------------- symmetric DxD helpers -- */

/* SymmProps<Symmetric>::getIndex (linal/Symmetry.hpp:40-46) */
static int og_sym_index(int D, int i, int j) {
	return (i < j) ? i * D - ((i - 1) * i) / 2 + j - i
	               : j * D - ((j - 1) * j) / 2 + i - j;
}

typedef struct { double a[3][3]; } og_sym; /* stored full, kept symmetric */

/* linal::symmDirectProduct (functions.hpp:546-558): (v1_i v2_j + v2_i v1_j)/2 */
static og_sym og_sdp(int D, const double* v1, const double* v2) {
	og_sym r;
	memset(&r, 0, sizeof(r));
	for (int i = 0; i < D; i++)
		for (int j = 0; j <= i; j++) {
			double x = (v1[i] * v2[j] + v2[i] * v1[j]) / 2;
			r.a[i][j] = x;
			r.a[j][i] = x;
		}
	return r;
}

static og_sym og_sym_scale(int D, og_sym m, double x) { /* m * x (operators.hpp:224-232) */
	for (int i = 0; i < D; i++) for (int j = 0; j < D; j++) m.a[i][j] = m.a[i][j] * x;
	return m;
}
static og_sym og_sym_div(int D, og_sym m, double x) { /* m / x (operators.hpp:257-265) */
	for (int i = 0; i < D; i++) for (int j = 0; j < D; j++) m.a[i][j] = m.a[i][j] / x;
	return m;
}
static og_sym og_sym_add(int D, og_sym a, og_sym b) {
	for (int i = 0; i < D; i++) for (int j = 0; j < D; j++) a.a[i][j] = a.a[i][j] + b.a[i][j];
	return a;
}
static og_sym og_sym_sub(int D, og_sym a, og_sym b) {
	for (int i = 0; i < D; i++) for (int j = 0; j < D; j++) a.a[i][j] = a.a[i][j] - b.a[i][j];
	return a;
}
static og_sym og_sym_neg(int D, og_sym a) {
	for (int i = 0; i < D; i++) for (int j = 0; j < D; j++) a.a[i][j] = -a.a[i][j];
	return a;
}
static og_sym og_sym_identity(int D) {
	og_sym r;
	memset(&r, 0, sizeof(r));
	for (int i = 0; i < D; i++) r.a[i][i] = 1;
	return r;
}
/* ElasticModel::correctFromTensorToVector (ElasticModel.hpp:321-327):
 * 2*s - Diag(s) */
static og_sym og_correct(int D, og_sym s) {
	og_sym r;
	memset(&r, 0, sizeof(r));
	for (int i = 0; i < D; i++)
		for (int j = 0; j < D; j++) {
			double d = (i == j) ? s.a[i][i] : 0.0;
			r.a[i][j] = (s.a[i][j] * 2) - d;
		}
	return r;
}

/* VelocitySigmaVariables::setVelocity / setSigma (VelocitySigmaVariables.hpp:45-70) */
static void og_set_velocity(int D, double* vec, const double* v) {
	for (int i = 0; i < D; i++) vec[i] = v[i];
}
static void og_set_sigma(int D, double* vec, og_sym s) {
	for (int i = 0; i < D; i++)
		for (int j = 0; j <= i; j++) vec[D + og_sym_index(D, i, j)] = s.a[i][j];
}
static og_sym og_get_sigma(int D, const double* vec) {
	og_sym r;
	memset(&r, 0, sizeof(r));
	for (int i = 0; i < D; i++)
		for (int j = 0; j <= i; j++) {
			r.a[i][j] = vec[D + og_sym_index(D, i, j)];
			r.a[j][i] = r.a[i][j];
		}
	return r;
}

/* --------------------------------------------------- local basis (axis) -- */

/* linal::createLocalBasis (basis.hpp:49-65) for n = e_axis, with
 * perpendicularClockwise (geometry.hpp:35-52) and crossProduct
 * (geometry.hpp:13-17).  basis[r][c], columns are (tau1, tau2, n). */
static void og_local_basis(int D, int axis, double basis[3][3]) {
	double n[3] = {0, 0, 0};
	n[axis] = 1;
	memset(basis, 0, sizeof(double) * 9);
	if (D == 1) {
		basis[0][0] = n[0];
	} else if (D == 2) {
		double tau[2] = {n[1], -n[0]};
		basis[0][0] = tau[0]; basis[0][1] = n[0];
		basis[1][0] = tau[1]; basis[1][1] = n[1];
	} else {
		double ans[3] = {n[1], -n[0], 0};
		if (n[0] == 0 && n[1] == 0) { ans[0] = n[2]; ans[1] = 0; ans[2] = 0; }
		double lv = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
		double la = sqrt(ans[0] * ans[0] + ans[1] * ans[1] + ans[2] * ans[2]);
		double t1[3], t2[3];
		for (int i = 0; i < 3; i++) t1[i] = (ans[i] * lv) / la;
		t2[0] = n[1] * t1[2] - n[2] * t1[1];
		t2[1] = n[2] * t1[0] - n[0] * t1[2];
		t2[2] = n[0] * t1[1] - n[1] * t1[0];
		for (int r = 0; r < 3; r++) {
			basis[r][0] = t1[r]; basis[r][1] = t2[r]; basis[r][2] = n[r];
		}
	}
}

/* --------------------------------------------- isotropic elastic matrices -- */

/* ElasticModel<D>::constructGcmMatrix + constructEigenvectors +
 * constructEigenstrings (ElasticModel.hpp:362-553), l = 1. */
static void og_construct_gcm_matrix(int D, double rho, double lambda, double mu,
                                    double basis[3][3],
                                    double* U, double* U1, double* L) {
	const int M = D + D * (D + 1) / 2;
	const double c1 = sqrt((lambda + 2 * mu) / rho);
	const double c2 = sqrt(mu / rho);
	const double l = 1;

	memset(U, 0, sizeof(double) * M * M);
	memset(U1, 0, sizeof(double) * M * M);
	memset(L, 0, sizeof(double) * M);

	/* L (ElasticModel.hpp:401-407) */
	L[0] = l * c1;
	L[1] = -l * c1;
	for (int i = 1; i < D; i++) {
		L[2 * i] = l * c2;
		L[2 * i + 1] = -l * c2;
	}

	/* n[i] = basis column (i + D - 1) % D */
	double n[3][3];
	for (int i = 0; i < D; i++) {
		int col = (i + D - 1) % D;
		for (int r = 0; r < D; r++) n[i][r] = basis[r][col];
	}
	const og_sym I = og_sym_identity(D);
	og_sym N[3][3];
	for (int i = 0; i < D; i++)
		for (int j = 0; j <= i; j++) {
			N[i][j] = og_sdp(D, n[i], n[j]);
			N[j][i] = N[i][j];
		}

	double vec[OG_MAXM];
	double tmpv[3];

	/* ---- U1: eigenvectors in columns (ElasticModel.hpp:416-483) */
	const double alpha = 0.5;
	memset(vec, 0, sizeof(vec));
	for (int r = 0; r < D; r++) tmpv[r] = n[0][r] * alpha;
	og_set_velocity(D, vec, tmpv);
	{
		og_sym t = og_sym_add(D, og_sym_scale(D, I, lambda),
		                      og_sym_scale(D, N[0][0], 2 * mu));
		og_set_sigma(D, vec, og_sym_scale(D, t, -alpha / c1));
	}
	for (int r = 0; r < M; r++) U1[r * M + 0] = vec[r];
	og_set_sigma(D, vec, og_sym_neg(D, og_get_sigma(D, vec)));
	for (int r = 0; r < M; r++) U1[r * M + 1] = vec[r];
	for (int i = 1; i < D; i++) {
		for (int r = 0; r < D; r++) tmpv[r] = n[i][r] * alpha;
		og_set_velocity(D, vec, tmpv);
		og_set_sigma(D, vec, og_sym_scale(D, N[0][i], -2 * alpha * mu / c2));
		for (int r = 0; r < M; r++) U1[r * M + 2 * i] = vec[r];
		og_set_sigma(D, vec, og_sym_neg(D, og_get_sigma(D, vec)));
		for (int r = 0; r < M; r++) U1[r * M + 2 * i + 1] = vec[r];
	}
	tmpv[0] = tmpv[1] = tmpv[2] = 0;
	og_set_velocity(D, vec, tmpv);
	if (D == 3) {
		og_set_sigma(D, vec, og_sym_scale(D, N[1][2], 2));
		for (int r = 0; r < M; r++) U1[r * M + 6] = vec[r];
		og_set_sigma(D, vec, og_sym_div(D, og_sym_sub(D, N[1][1], N[2][2]), 2));
		for (int r = 0; r < M; r++) U1[r * M + 7] = vec[r];
		og_set_sigma(D, vec, og_sym_div(D, og_sym_add(D, N[1][1], N[2][2]), 2));
		for (int r = 0; r < M; r++) U1[r * M + 8] = vec[r];
	} else if (D == 2) {
		og_set_sigma(D, vec, og_sym_sub(D, I, N[0][0]));
		for (int r = 0; r < M; r++) U1[r * M + 4] = vec[r];
	}

	/* ---- U: eigenstrings in rows (ElasticModel.hpp:486-553) */
	memset(vec, 0, sizeof(vec));
	og_set_velocity(D, vec, n[0]);
	og_set_sigma(D, vec, og_correct(D, og_sym_div(D, N[0][0], -c1 * rho)));
	for (int c = 0; c < M; c++) U[0 * M + c] = vec[c];
	og_set_sigma(D, vec, og_sym_neg(D, og_get_sigma(D, vec)));
	for (int c = 0; c < M; c++) U[1 * M + c] = vec[c];
	for (int i = 1; i < D; i++) {
		og_set_velocity(D, vec, n[i]);
		og_set_sigma(D, vec, og_correct(D, og_sym_div(D, N[0][i], -c2 * rho)));
		for (int c = 0; c < M; c++) U[(2 * i) * M + c] = vec[c];
		og_set_sigma(D, vec, og_sym_neg(D, og_get_sigma(D, vec)));
		for (int c = 0; c < M; c++) U[(2 * i + 1) * M + c] = vec[c];
	}
	og_set_velocity(D, vec, tmpv);
	if (D == 3) {
		og_set_sigma(D, vec, og_correct(D, N[1][2]));
		for (int c = 0; c < M; c++) U[6 * M + c] = vec[c];
		og_set_sigma(D, vec, og_correct(D, og_sym_sub(D, N[1][1], N[2][2])));
		for (int c = 0; c < M; c++) U[7 * M + c] = vec[c];
		og_sym t = og_sym_sub(D, og_sym_add(D, N[1][1], N[2][2]),
		                      og_sym_scale(D, N[0][0], 2 * lambda / (lambda + 2 * mu)));
		og_set_sigma(D, vec, og_correct(D, t));
		for (int c = 0; c < M; c++) U[8 * M + c] = vec[c];
	} else if (D == 2) {
		og_sym t = og_sym_sub(D, N[1][1],
		                      og_sym_scale(D, N[0][0], lambda / (lambda + 2 * mu)));
		og_set_sigma(D, vec, og_correct(D, t));
		for (int c = 0; c < M; c++) U[4 * M + c] = vec[c];
	}
}

int og_isotropic_elastic_matrices(int D, double rho, double lambda, double mu,
                                  double* U, double* U1, double* L) {
	if (D < 1 || D > 3) return -1;
	if (!(rho > 0) || !(mu > 0)) return -1;
	const int M = D + D * (D + 1) / 2;
	for (int s = 0; s < D; s++) {
		double basis[3][3];
		og_local_basis(D, s, basis);
		og_construct_gcm_matrix(D, rho, lambda, mu, basis,
		                        U + (size_t)s * M * M, U1 + (size_t)s * M * M,
		                        L + (size_t)s * M);
	}
	return 0;
}

/* ----------------------------------------------------------- interpolate -- */

/* EqualDistanceLineInterpolator::interpolate (hpp:56-71). */
int og_interpolate(int n, int M, double* src, double q, double* out) {
	const int p = n - 1;
	for (int c = 0; c < M; c++) out[c] = src[c];
	for (int i = 1; i <= p; i++) {
		const double coef = ((q - i) + 1) / i;
		for (int j = 0; j < p - i + 1; j++)
			for (int c = 0; c < M; c++)
				src[j * M + c] = (src[(j + 1) * M + c] - src[j * M + c]) * coef;
		for (int c = 0; c < M; c++) out[c] += src[c];
	}
	return 0;
}

/* EqualDistanceLineInterpolator::minMaxInterpolate (hpp:18-43).  The
 * reference reads src[k+1] past the vector end when floor(q) == n-1; that is
 * undefined behaviour there, so it is reported as an error here. */
int og_min_max_interpolate(int n, int M, double* src, double q, double* out) {
	if (!(q >= 0)) return -1;
	const size_t k = (size_t)q;
	if (k > (size_t)(n - 1)) return -1;
	if (k + 1 > (size_t)(n - 1)) return -1; /* UB read in the reference */
	double mx[OG_MAXM], mn[OG_MAXM];
	for (int c = 0; c < M; c++) {
		mx[c] = fmax(src[k * M + c], src[(k + 1) * M + c]);
		mn[c] = fmin(src[k * M + c], src[(k + 1) * M + c]);
	}
	og_interpolate(n, M, src, q, out);
	for (int c = 0; c < M; c++) {
		if (out[c] > mx[c]) out[c] = mx[c];
		else if (out[c] < mn[c]) out[c] = mn[c];
	}
	return 0;
}

/* ------------------------------------------------------------- products -- */

void og_diagonal_multiply(int M, const double* A, const double* B, double* r) {
	for (int i = 0; i < M; i++) {
		double acc = A[i * M + 0] * B[0 * M + i];
		for (int j = 1; j < M; j++) acc += A[i * M + j] * B[j * M + i];
		r[i] = acc;
	}
}

void og_local_gcm_step(int M, const double* U1, const double* U,
                       const double* V, double* out) {
	double r[OG_MAXM];
	og_diagonal_multiply(M, U, V, r);
	for (int i = 0; i < M; i++) {
		double acc = U1[i * M + 0] * r[0];
		for (int n = 1; n < M; n++) acc += U1[i * M + n] * r[n];
		out[i] = acc;
	}
}

/* ------------------------------------------------------------ the stage -- */

static int og_interp_around(const og_grid* g, const long long im[3],
                            const double* pde, int s, long long idx,
                            const double* dx, double* V) {
	const int M = g->M, n = g->bs + 1;
	double src[(OG_MAXBS + 1) * OG_MAXM];
	double col[OG_MAXM];
	for (int k = 0; k < M; k++) {
		const long long shift = (dx[k] > 0) ? 1 : -1;
		for (int i = 0; i < n; i++) {
			const double* p = pde + (idx + shift * i * im[s]) * M;
			for (int c = 0; c < M; c++) src[i * M + c] = p[c];
		}
		if (og_min_max_interpolate(n, M, src, fabs(dx[k]) / g->h[s], col)) return -1;
		for (int c = 0; c < M; c++) V[c * M + k] = col[c];
	}
	return 0;
}

int og_interpolate_values_around(const og_grid* g, const double* pde, int s,
                                 const int it[3], const double* dx, double* V) {
	long long im[3];
	og_index_maker(g, im);
	return og_interp_around(g, im, pde, s, og_get_index(g, im, it), dx, V);
}

int og_stage(const og_grid* g, int s, double tau, const double* cur,
             double* next, const uint8_t* mat_id, const double* U,
             const double* U1, const double* L, int nthreads) {
	const int D = g->D, M = g->M;
	if (M > OG_MAXM || g->bs > OG_MAXBS || s < 0 || s >= D) return -1;
	long long im[3];
	og_index_maker(g, im);
	const int X = g->sizes[0];
	const int Y = D > 1 ? g->sizes[1] : 1;
	const int Z = D > 2 ? g->sizes[2] : 1;
	int err = 0;
	(void)nthreads;
#ifdef _OPENMP
	if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) reduction(| : err)
#endif
	for (int x = 0; x < X; x++) {
		double dx[OG_MAXM], V[OG_MAXM * OG_MAXM], out[OG_MAXM];
		for (int y = 0; y < Y; y++)
			for (int z = 0; z < Z; z++) {
				int it[3] = {x, y, z};
				const long long idx = og_get_index(g, im, it);
				const int m = mat_id ? mat_id[idx] : 0;
				const double* Um = U + ((size_t)m * D + s) * M * M;
				const double* U1m = U1 + ((size_t)m * D + s) * M * M;
				const double* Lm = L + ((size_t)m * D + s) * M;
				/* crossingPoints: -timeStep * diag(L) (hpp:56-59) */
				for (int k = 0; k < M; k++) dx[k] = Lm[k] * (-tau);
				if (og_interp_around(g, im, cur, s, idx, dx, V)) { err |= 1; continue; }
				og_local_gcm_step(M, U1m, Um, V, out);
				for (int c = 0; c < M; c++) next[idx * M + c] = out[c];
			}
	}
	return err ? -1 : 0;
}

/* ---------------------------------------------------------------- random -- */

double og_splitmix_uniform(uint64_t seed, uint64_t n) {
	uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	z = z ^ (z >> 31);
	return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

void og_fill_random(const og_grid* g, const int gsizes[3], uint64_t seed,
                    double* pde) {
	const int D = g->D, M = g->M;
	long long im[3];
	og_index_maker(g, im);
	const int X = g->sizes[0];
	const int Y = D > 1 ? g->sizes[1] : 1;
	const int Z = D > 2 ? g->sizes[2] : 1;
	const uint64_t GY = D > 1 ? (uint64_t)gsizes[1] : 1;
	const uint64_t GZ = D > 2 ? (uint64_t)gsizes[2] : 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
	for (int x = 0; x < X; x++)
		for (int y = 0; y < Y; y++)
			for (int z = 0; z < Z; z++) {
				int it[3] = {x, y, z};
				const long long idx = og_get_index(g, im, it);
				const uint64_t gx = (uint64_t)(x + g->start[0]);
				const uint64_t gy = D > 1 ? (uint64_t)(y + g->start[1]) : 0;
				const uint64_t gz = D > 2 ? (uint64_t)(z + g->start[2]) : 0;
				const uint64_t base = ((gx * GY + gy) * GZ + gz) * (uint64_t)M;
				for (int c = 0; c < M; c++)
					pde[idx * M + c] = og_splitmix_uniform(seed, base + (uint64_t)c);
			}
}
