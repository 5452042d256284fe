// elastic_model.hpp -- host-side GcmMatrices for isotropic elastic media.
//
// Mirrors rheology/models/ElasticModel.hpp:57-65, 362-553 (constructGcmMatrices,
// constructGcmMatrix, constructEigenvectors, constructEigenstrings) for the
// identity calculation basis the cubic engine uses.  Built once per material on
// the host; the device only ever sees the finished U / U1 / L tables.  Every
// expression keeps the reference's evaluation order so the tables are bitwise
// the reference's (checked against the oracle in tests/test_abi.py::test_host_matrices_match_oracle_bitwise).
#pragma once

#include <array>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <type_traits>

namespace gcm {

using real = double;

constexpr int pdeSize(int D) { return D + D * (D + 1) / 2; }

/// Isotropic material (rheology/materials/IsotropicMaterial.hpp:7-27).
struct IsotropicMaterial {
	real rho = 0, lambda = 0, mu = 0;
	real yieldStrength = 0;             ///< plasticity parameter
	real continualDamageParameter = 0;  ///< parameter in the continual damage equation
	int materialNumber = 0;
	real tau0 = 0;                      ///< viscosity parameter (decay time), MaxwellViscosityOde
	IsotropicMaterial() = default;
	IsotropicMaterial(real rho_, real lambda_, real mu_, real yieldStrength_ = 0,
	                  real continualDamageParameter_ = 0, int materialNumber_ = 0, real tau0_ = 0)
	    : rho(rho_), lambda(lambda_), mu(mu_), yieldStrength(yieldStrength_),
	      continualDamageParameter(continualDamageParameter_), materialNumber(materialNumber_),
	      tau0(tau0_) {}
};

/// GcmMatrices<M,D>::GcmMatrix (util/math/GridCharacteristicMethod.hpp:40-52), row-major.
template <int D>
struct GcmMatrices {
	static constexpr int M = pdeSize(D);
	struct GcmMatrix {
		std::array<real, M * M> U{}, U1{};
		std::array<real, M> L{};
		real getMaximalEigenvalue() const {
			real ans = 0;
			for (int i = 0; i < M; i++) ans = std::fmax(ans, std::fabs(L[i]));
			return ans;
		}
	};
	GcmMatrix m[D];
	real getMaximalEigenvalue() const {
		real ans = 0;
		for (int i = 0; i < D; i++) ans = std::fmax(ans, m[i].getMaximalEigenvalue());
		return ans;
	}
};

namespace detail {

/// Symmetric DxD tensor kept in full storage (linal::SymmetricMatrix).
template <int D>
struct Sym {
	real a[D][D] = {};
	Sym operator*(real x) const {  // m * x  (linal/operators.hpp:224-232)
		Sym r;
		for (int i = 0; i < D; i++)
			for (int j = 0; j < D; j++) r.a[i][j] = a[i][j] * x;
		return r;
	}
	Sym operator/(real x) const {  // m / x  (linal/operators.hpp:257-265)
		Sym r;
		for (int i = 0; i < D; i++)
			for (int j = 0; j < D; j++) r.a[i][j] = a[i][j] / x;
		return r;
	}
	Sym operator+(const Sym& o) const {
		Sym r;
		for (int i = 0; i < D; i++)
			for (int j = 0; j < D; j++) r.a[i][j] = a[i][j] + o.a[i][j];
		return r;
	}
	Sym operator-(const Sym& o) const {
		Sym r;
		for (int i = 0; i < D; i++)
			for (int j = 0; j < D; j++) r.a[i][j] = a[i][j] - o.a[i][j];
		return r;
	}
	Sym operator-() const {
		Sym r;
		for (int i = 0; i < D; i++)
			for (int j = 0; j < D; j++) r.a[i][j] = -a[i][j];
		return r;
	}
	static Sym identity() {
		Sym r;
		for (int i = 0; i < D; i++) r.a[i][i] = 1;
		return r;
	}
};

template <int D>
Sym<D> operator*(real x, const Sym<D>& m) { return m * x; }  // operators.hpp:243-246

/// linal::symmDirectProduct (linal/functions.hpp:546-558)
template <int D>
Sym<D> symmDirectProduct(const real* v1, const real* v2) {
	Sym<D> r;
	for (int i = 0; i < D; i++)
		for (int j = 0; j <= i; j++) {
			const real x = (v1[i] * v2[j] + v2[i] * v1[j]) / 2;
			r.a[i][j] = x;
			r.a[j][i] = x;
		}
	return r;
}

/// ElasticModel::correctFromTensorToVector: 2 * s - Diag(s) (ElasticModel.hpp:321-327)
template <int D>
Sym<D> correctFromTensorToVector(const Sym<D>& s) {
	Sym<D> r;
	for (int i = 0; i < D; i++)
		for (int j = 0; j < D; j++) r.a[i][j] = (s.a[i][j] * 2) - (i == j ? s.a[i][i] : 0.0);
	return r;
}

/// Position of sigma(i,j) in the PDE vector (VelocitySigmaVariables.hpp:82-96,
/// SymmProps<Symmetric>::getIndex, linal/Symmetry.hpp:40-46).
constexpr int sigmaIndex(int D, int i, int j) {
	return D + ((i < j) ? i * D - ((i - 1) * i) / 2 + j - i : j * D - ((j - 1) * j) / 2 + i - j);
}

template <int D>
struct PdeVec {
	real v[pdeSize(D)] = {};
	void setVelocity(const real* x) {
		for (int i = 0; i < D; i++) v[i] = x[i];
	}
	void setSigma(const Sym<D>& s) {
		for (int i = 0; i < D; i++)
			for (int j = 0; j <= i; j++) v[sigmaIndex(D, i, j)] = s.a[i][j];
	}
	Sym<D> getSigma() const {
		Sym<D> s;
		for (int i = 0; i < D; i++)
			for (int j = 0; j <= i; j++) s.a[i][j] = s.a[j][i] = v[sigmaIndex(D, i, j)];
		return s;
	}
};

/// linal::createLocalBasis(n) (linal/basis.hpp:49-65) with
/// perpendicularClockwise (linal/geometry.hpp:35-52); columns (tau1, tau2, n).
template <int D>
void localBasisOf(const real nIn[D], real basis[D][D]) {
	real n[3] = {0, 0, 0};
	for (int i = 0; i < D; i++) n[i] = nIn[i];
	if constexpr (D == 1) {
		basis[0][0] = n[0];
	} else if constexpr (D == 2) {
		const real tau[2] = {n[1], -n[0]};
		basis[0][0] = tau[0];
		basis[0][D - 1] = n[0];
		basis[1][0] = tau[1];
		basis[1][D - 1] = n[1];
	} else {
		real ans[3] = {n[1], -n[0], 0};
		if (n[0] == 0 && n[1] == 0) {
			ans[0] = n[2];
			ans[1] = 0;
			ans[2] = 0;
		}
		const real lv = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
		const real la = std::sqrt(ans[0] * ans[0] + ans[1] * ans[1] + ans[2] * ans[2]);
		real t1[3], t2[3];
		for (int i = 0; i < 3; i++) t1[i] = (ans[i] * lv) / la;
		t2[0] = n[1] * t1[2] - n[2] * t1[1];  // crossProduct (linal/geometry.hpp:13-17)
		t2[1] = n[2] * t1[0] - n[0] * t1[2];
		t2[2] = n[0] * t1[1] - n[1] * t1[0];
		for (int r = 0; r < D; r++) {
			basis[r][0] = t1[r];
			basis[r][1 % D] = t2[r];
			basis[r][D - 1] = n[r];
		}
	}
}

/// createLocalBasis(e_axis)
template <int D>
void localBasis(int axis, real basis[D][D]) {
	real n[D] = {};
	n[axis] = 1;
	localBasisOf<D>(n, basis);
}

}  // namespace detail

/// ElasticModel<D> (rheology/models/ElasticModel.hpp) -- matrix construction only.
template <int D>
struct ElasticModel {
	static constexpr int DIMENSIONALITY = D;
	static constexpr int PDE_SIZE = pdeSize(D);
	using Matrices = GcmMatrices<D>;

	/// constructGcmMatrices with the identity basis (ElasticModel.hpp:57-65)
	static void constructGcmMatrices(Matrices& out, const IsotropicMaterial& mat) {
		if (!(mat.rho > 0) || !(mat.mu > 0))
			throw std::invalid_argument("isotropic material needs rho > 0 and mu > 0");
		for (int i = 0; i < D; i++) {
			real basis[D][D] = {};
			detail::localBasis<D>(i, basis);
			constructGcmMatrix(out.m[i], mat, basis);
		}
	}

	/// constructGcmMatrices with an arbitrary calculation basis: stage i along
	/// column i of `calc` (ElasticModel.hpp:57-65).
	static void constructGcmMatrices(Matrices& out, const IsotropicMaterial& mat,
	                                 const real calc[D][D]) {
		if (!(mat.rho > 0) || !(mat.mu > 0))
			throw std::invalid_argument("isotropic material needs rho > 0 and mu > 0");
		for (int i = 0; i < D; i++) {
			real n[D], basis[D][D] = {};
			for (int r = 0; r < D; r++) n[r] = calc[r][i];
			detail::localBasisOf<D>(n, basis);
			constructGcmMatrix(out.m[i], mat, basis);
		}
	}

	/// constructGcmMatrix + constructEigenvectors + constructEigenstrings
	/// (ElasticModel.hpp:362-553), scale l = 1.
	static void constructGcmMatrix(typename Matrices::GcmMatrix& m, const IsotropicMaterial& mat,
	                               const real basis[D][D]) {
		using detail::Sym;
		constexpr int M = PDE_SIZE;
		const real rho = mat.rho, lambda = mat.lambda, mu = mat.mu;
		const real c1 = std::sqrt((lambda + 2 * mu) / rho);
		const real c2 = std::sqrt(mu / rho);
		const real l = 1;
		m.U.fill(0);
		m.U1.fill(0);
		m.L.fill(0);
		m.L[0] = l * c1;
		m.L[1] = -l * c1;
		for (int i = 1; i < D; i++) {
			m.L[2 * i] = l * c2;
			m.L[2 * i + 1] = -l * c2;
		}
		real n[D][D];
		for (int i = 0; i < D; i++)
			for (int r = 0; r < D; r++) n[i][r] = basis[r][(i + D - 1) % D];
		const Sym<D> I = Sym<D>::identity();
		Sym<D> N[D][D];
		for (int i = 0; i < D; i++)
			for (int j = 0; j <= i; j++) N[i][j] = N[j][i] = detail::symmDirectProduct<D>(n[i], n[j]);

		auto setCol = [&](int c, const detail::PdeVec<D>& v) {
			for (int r = 0; r < M; r++) m.U1[r * M + c] = v.v[r];
		};
		auto setRow = [&](int r, const detail::PdeVec<D>& v) {
			for (int c = 0; c < M; c++) m.U[r * M + c] = v.v[c];
		};
		real zero[D] = {};
		real tmp[D];

		// ---- eigenvectors (columns of U1), ElasticModel.hpp:416-483
		const real alpha = 0.5;
		detail::PdeVec<D> vec;
		for (int r = 0; r < D; r++) tmp[r] = n[0][r] * alpha;  // alpha * n[0]
		vec.setVelocity(tmp);
		vec.setSigma(-alpha / c1 * (lambda * I + 2 * mu * N[0][0]));
		setCol(0, vec);
		vec.setSigma(-vec.getSigma());
		setCol(1, vec);
		for (int i = 1; i < D; i++) {
			for (int r = 0; r < D; r++) tmp[r] = n[i][r] * alpha;
			vec.setVelocity(tmp);
			vec.setSigma(-2 * alpha * mu / c2 * N[0][i]);
			setCol(2 * i, vec);
			vec.setSigma(-vec.getSigma());
			setCol(2 * i + 1, vec);
		}
		vec.setVelocity(zero);
		if constexpr (D == 3) {
			vec.setSigma(2 * N[1][D - 1]);
			setCol(6, vec);
			vec.setSigma((N[1][1] - N[D - 1][D - 1]) / 2);
			setCol(7, vec);
			vec.setSigma((N[1][1] + N[D - 1][D - 1]) / 2);
			setCol(8, vec);
		} else if constexpr (D == 2) {
			vec.setSigma(I - N[0][0]);
			setCol(4, vec);
		}

		// ---- eigenstrings (rows of U), ElasticModel.hpp:486-553
		detail::PdeVec<D> row;
		row.setVelocity(n[0]);
		row.setSigma(detail::correctFromTensorToVector(N[0][0] / (-c1 * rho)));
		setRow(0, row);
		row.setSigma(-row.getSigma());
		setRow(1, row);
		for (int i = 1; i < D; i++) {
			row.setVelocity(n[i]);
			row.setSigma(detail::correctFromTensorToVector(N[0][i] / (-c2 * rho)));
			setRow(2 * i, row);
			row.setSigma(-row.getSigma());
			setRow(2 * i + 1, row);
		}
		row.setVelocity(zero);
		if constexpr (D == 3) {
			row.setSigma(detail::correctFromTensorToVector(N[1][D - 1]));
			setRow(6, row);
			row.setSigma(detail::correctFromTensorToVector(N[1][1] - N[D - 1][D - 1]));
			setRow(7, row);
			row.setSigma(detail::correctFromTensorToVector(
			    N[1][1] + N[D - 1][D - 1] - 2 * lambda / (lambda + 2 * mu) * N[0][0]));
			setRow(8, row);
		} else if constexpr (D == 2) {
			row.setSigma(detail::correctFromTensorToVector(
			    N[1][1] - lambda / (lambda + 2 * mu) * N[0][0]));
			setRow(4, row);
		}
	}
};

}  // namespace gcm
