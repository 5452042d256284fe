// host_capi.cpp -- C entry points of the host mirror used by the Python side.
#include "elastic_model.hpp"

extern "C" {

/// ElasticModel<D>::constructGcmMatrices for an isotropic material, identity
/// basis: U, U1 [D][M*M] row-major, L [D][M].  Returns 0 or -1 (bad input).
int gcm_host_isotropic_elastic_matrices(int D, double rho, double lambda, double mu, double* U,
                                        double* U1, double* L) {
	try {
		auto run = [&](auto tag) {
			constexpr int DD = decltype(tag)::value;
			constexpr int M = gcm::pdeSize(DD);
			gcm::GcmMatrices<DD> m;
			gcm::ElasticModel<DD>::constructGcmMatrices(m, gcm::IsotropicMaterial(rho, lambda, mu));
			for (int s = 0; s < DD; s++) {
				for (int i = 0; i < M * M; i++) {
					U[s * M * M + i] = m.m[s].U[i];
					U1[s * M * M + i] = m.m[s].U1[i];
				}
				for (int k = 0; k < M; k++) L[s * M + k] = m.m[s].L[k];
			}
		};
		switch (D) {
		case 1: run(std::integral_constant<int, 1>()); return 0;
		case 2: run(std::integral_constant<int, 2>()); return 0;
		case 3: run(std::integral_constant<int, 3>()); return 0;
		default: return -1;
		}
	} catch (...) {
		return -1;
	}
}

}
