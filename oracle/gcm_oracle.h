/*
 * gcm_oracle.h -- CPU restatement of libgcm's cubic grid-characteristic
 * stage path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker.  The product (gcm_amd/,
 * libgcmx.so) never links, loads or calls anything under oracle/.
 *
 * Parity status: pinned against the reference's own known-answer tests
 * (TestInterpolator.cpp, TestGridCharacteristicMethod.cpp, TestLinal.cpp,
 * TestCubicGrid.cpp, TestGcmMatrices.cpp) and the bitwise sanity anchors the
 * survey measured with the reference itself:
 * see tests/test_oracle.py.  The reference cannot be compiled here without
 * generated headers and library stand-ins, so no
 * oracle/_ref build exists.
 *
 * Memory layout: exactly the reference's DefaultMesh storage -- an AoS array
 * of `M` doubles per node over ALL nodes including ghosts, indexed by
 * CubicGrid::getIndex (X slowest, last axis fastest).
 */
#ifndef GCM_ORACLE_H
#define GCM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct og_grid {
	int D;          /* dimensionality 1..3 */
	int M;          /* PDE size: D + D(D+1)/2 */
	int bs;         /* borderSize (ghost layers) */
	int sizes[3];
	int start[3];
	double h[3];
} og_grid;

/* CubicGrid::calculateIndexMaker / sizeOfAllNodes (CubicGrid.hpp:132-134, 202-225) */
void   og_index_maker(const og_grid* g, long long im[3]);
long long og_size_of_all_nodes(const og_grid* g);

/* ElasticModel<D>::constructGcmMatrices with the identity basis
 * (ElasticModel.hpp:57-65, 362-553).  Outputs per axis s:
 *   U [s*M*M + i*M + j], U1 [same], L [s*M + k]. */
int og_isotropic_elastic_matrices(int D, double rho, double lambda, double mu,
                                  double* U, double* U1, double* L);

/* EqualDistanceLineInterpolator::interpolate / minMaxInterpolate
 * (EqualDistanceLineInterpolator.hpp:18-71).  src is (n) vectors of M
 * doubles, row-major, and is OVERWRITTEN like the reference.  Returns 0, or
 * -1 where the reference would throw (q < 0 or floor(q) > n-1). */
int og_interpolate(int n, int M, double* src, double q, double* out);
int og_min_max_interpolate(int n, int M, double* src, double q, double* out);

/* linal::diagonalMultiply and operator* (functions.hpp:254-267,
 * operators.hpp:109-123), then localGcmStep
 * (util/math/GridCharacteristicMethod.hpp:10-17). Matrices row-major MxM. */
void og_diagonal_multiply(int M, const double* A, const double* B, double* r);
void og_local_gcm_step(int M, const double* U1, const double* U,
                       const double* V, double* out);

/* GridCharacteristicMethod<Mesh>::interpolateValuesAround
 * (engine/cubic/GridCharacteristicMethod.hpp:73-87): V is MxM row-major,
 * column k = interpolated PDE vector for shift dx[k].  Returns 0 or -1. */
int og_interpolate_values_around(const og_grid* g, const double* pde, int s,
                                 const int it[3], const double* dx, double* V);

/* GridCharacteristicMethod<Mesh>::stage (GridCharacteristicMethod.hpp:42-52)
 * over all inner nodes: next(it) = localGcmStep(U1, U, interp(...)).
 * mat_id: NULL (one material, table index 0) or one byte per node of the
 * all-nodes array.  Tables: U/U1 [mat][D][M*M], L [mat][D][M].
 * nthreads: OpenMP threads (<=0: library default).  Returns 0 or -1 (a
 * reference assertion would have thrown). */
int og_stage(const og_grid* g, int s, double tau, const double* cur,
             double* next, const uint8_t* mat_id, const double* U,
             const double* U1, const double* L, int nthreads);

/* Parity-random field (SURVEY.md §8d "parity-random"): every component of
 * every INNER node = uniform [-1,1) from SplitMix64(seed) indexed in global
 * (x,y,z,c) order over a global box of `gsizes`; ghosts left untouched. */
void og_fill_random(const og_grid* g, const int gsizes[3], uint64_t seed,
                    double* pde);
double og_splitmix_uniform(uint64_t seed, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
