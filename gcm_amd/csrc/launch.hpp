// launch.hpp -- host-side launchers exported by the kernel translation units.
#pragma once

#include "common.hpp"

#include <string>

namespace gcmx {

// gcmx.hip: gcmx_last_error() of the calling thread (shared by every ABI file).
void set_last_error(const std::string& msg);

// kernels_generic.hip
bool launch_stage_generic(const double* cur, double* nxt, const Geo& g, int s,
                          const AxisTable* tabs, const uint8_t* mat, hipStream_t st);
void launch_fill_random(double* cur, const Geo& g, const int gstart[3], long long GY,
                        long long GZ, uint64_t seed, hipStream_t st);
void launch_copy_box(double* dst, const Geo& gd, const double* src, const Geo& gs,
                     const int dmin[3], const int smin[3], const int ext[3], hipStream_t st);
void launch_scale_stress(double* cur, const Geo& g, const uint8_t* mat_d, const double* f_d,
                         double f0, hipStream_t st);
// Per-material ODE factors by value (at most 255 materials).
struct OdeFactors {
	int n;
	double f[255];
};
void launch_set_factors(double* dst_d, const OdeFactors& v, hipStream_t st);
// The quantities of one cubic border condition, by value (kernel arguments):
// PhysicalQuantities codes and timeDependency(t), in the reference's map order.
constexpr int kMaxBorderQ = 16;
struct BorderQ {
	int n;
	int q[kMaxBorderQ];
	double v[kMaxBorderQ];
};
// BorderConditions::handleBorderPoint over a device-resident list of face nodes.
void launch_border_fill(double* cur, const Geo& g, int axis, int inner_sign, int n_nodes,
                        const int* nodes_d, const BorderQ& bq, hipStream_t st);
// The same over every node of the face (axis, side = -1 / +1).
void launch_face_fill(double* cur, const Geo& g, int axis, int side, const BorderQ& bq,
                      hipStream_t st);
// The same over a per-node face map (gcmx_face_map): node i of the face takes
// condition bq_d[map_d[i]], none when map_d[i] == kNoFaceCond (ghosts untouched).
void launch_face_fill_map(double* cur, const Geo& g, int axis, int side, const uint8_t* map_d,
                          const BorderQ* bq_d, hipStream_t st);


// kernels_fast.hip -- 3-D, homogeneous, structured isotropic-elastic matrices.
// Per-axis values the fast kernels receive by value (kernel arguments, i.e.
// scalar registers): the six material magnitudes of U / U1 and the Newton data
// of the two distinct |eigenvalues| (c1: feet 0,1; c2: feet 2..5).
struct IsoAxis {
	double a, b, g;      // U:  sigma_ss of rows 0/1, sigma_ts of rows 2..5, sigma_ss of row 8
	double p1, p2, s;    // U1: sigma_ss / sigma_tt of columns 0/1, sigma_st of columns 2..5
	double c1[3], c2[3]; // ((q - i) + 1) / i, i = 1..bs
	double w1[3], w2[3]; // the same interpolant's Lagrange weights (floor(q) = 0, bs <= 2; else 0):
	                     // sum_i w[i] s_i == Newton's s0 + c0 D1 + c0 c1 D2 (lagrange_weights)
	int kf1, kf2;        // floor(q)
};
// Lagrange weights w[0..bs] of the Newton interpolant with coefficients c
// (EqualDistanceLineInterpolator.hpp:56-71: ans = s0 + c0 (s1 - s0) + c0 c1 (s2 - 2 s1 + s0))
inline void lagrange_weights(const double* c, int bs, double* w) {
	w[0] = w[1] = w[2] = 0.0;
	if (bs == 1) {
		w[0] = 1.0 - c[0];
		w[1] = c[0];
	} else if (bs == 2) {
		const double c01 = c[0] * c[1];
		w[0] = (1.0 - c[0]) + c01;
		w[1] = c[0] - 2.0 * c01;
		w[2] = c01;
	}
}
bool iso_axis_extract(int s, const double* U, const double* U1, const double* L, IsoAxis& A);
// kernels_2d.hip: the one-pass 2-D step.  One material: tabs = its X and Y
// tables; iso = its two IsoAxis (the isotropic structure, iso2_axis_extract) or
// null.  borderSize 1..kStep2dMaxBs (the isotropic kernel up to 3), y ghost
// columns of both layers zero.
constexpr int kStep2dMaxBs = 5;
bool iso2_axis_extract(int s, const double* U, const double* U1, const double* L, IsoAxis& A);
bool step2d_supported(const Geo& g);
bool step2d_iso_supported(const Geo& g);
// Cubic border conditions on the two y faces of the 2-D step (face f: 0 y-,
// 1 y+), as the one pass forms them: the Y stage's ghost columns are the
// mirrored X results with the components in mask[f] set to -inner + two_v[f][c]
// (BorderConditions.hpp:94-114); the x faces are filled in memory before the
// launch.  Isotropic kernel only; needs Y >= bs + 1.
struct Face2 {
	unsigned on;       // bit f: face f has a condition
	unsigned mask[2];  // overridden components
	double two_v[2][5];
};
bool launch_step2d(const double* cur, double* nxt, const Geo& g, const AxisTable* tabs, const IsoAxis* iso,
                   hipStream_t st, const char** kname, const Face2* faces = nullptr);
bool fast_layout_ok(const Geo& g);     // the per-stage kernels: layer planes < 2^32 bytes
bool onepass_layout_ok(const Geo& g);  // the one-pass kernels: 32-bit offsets within a block's planes
bool launch_march(const double* cur, double* nxt, const Geo& g, int s, const IsoAxis& A,
                  int x0, int x1, hipStream_t st);
bool launch_line_z(const double* cur, double* nxt, const Geo& g, const IsoAxis& A, int x0,
                   int x1, hipStream_t st);
// The one-pass step needs 2*bs <= Z <= 1024 (one block spans a whole z row).
bool fused_supported(const Geo& g);
// One cubic border condition as the one-pass step applies it to a ghost: the
// components in `mask` set to -inner + two_v[c], the others mirrored
// (BorderConditions.hpp:94-114; two_v = 2 * timeDependency(t)).
struct FaceCond {
	unsigned mask;
	unsigned pad_;
	double two_v[9];
};
// Materials of the heterogeneous one-pass step: their tables live in LDS (more
// materials take the per-stage path).
constexpr int kHetMaxMaterials = 32;
constexpr int kMaxFaceConds = 8;  // conditions of one per-node face map (gcmx_face_map)
constexpr uint8_t kNoFaceCond = 255;
// Cubic border conditions on the y/z faces, as the one-pass step consumes
// them (face f: 0 y-, 1 y+, 2 z-, 3 z+): the ghosts are the mirrored inner nodes
// with the components in mask[f] set to -inner + two_v[f][c]
// (BorderConditions.hpp:94-114; two_v = 2 * timeDependency(t)).  A face with a
// per-node map (map[f] != null: PARTIAL faces, e.g. titan's cylinder,
// launcher/ndi.hpp:309-315) takes each face node's own condition
// conds[map[f][node]] instead -- the last condition whose area holds the node --
// and kNoFaceCond for a node no condition covers, whose ghosts stay zero (the
// reference never writes them); maps are [x][z] (y faces) / [x][y] (z faces)
// over the context's inner nodes.
struct FaceBC {
	unsigned on;          // bit f: face f has a condition
	unsigned mask[4];     // overridden components
	double two_v[4][9];
	// MaxwellViscosityOde folded into the store epilogue (gcmx_step_ode): every
	// stress component of the step's result times `ode` (Ode.hpp:28-37) when ode_on
	unsigned ode_on;
	double ode;
	const double* ode_f;  // HET: per-material factors (device, indexed by the node's id)
	const uint8_t* map[4];
	const FaceCond* conds;
};
// Condition tables of a face map into device memory, ordered on the stream.
struct FaceTables {
	int n;
	BorderQ bq[kMaxFaceConds];
	FaceCond fc[kMaxFaceConds];
};
void launch_set_face_tables(BorderQ* bq_d, FaceCond* fc_d, const FaceTables& t, hipStream_t st);
// The one-pass step with FaceBC face conditions (on != 0) needs bs <= 2, Z <= 512
// or the z split (then also zs_admissible) and Y, Z >= 2*bs + 2; a FaceBC with
// on == 0 carries only the ODE factor.
bool fused_faces_supported(const Geo& g);
// One pass per time step: X, Y, Z stages of planes [x0, x1), `a` = the three axes.
// `chunk`: y rows per block (0 = automatic, kernels_xyz.hip: xyz_chunk_for).
// `faces`: y/z face conditions and the ODE factor (null, or on == 0: y/z ghosts of
// both layers are zero); the ODE factor needs the k_step_tx2 path (bs <= 2, Z <= 512).
// Per-node materials for the one-pass step (k_step_tx2<..., HET>): per material
// one IsoAxis (the three axes' tables identical, floor(q) = 0), the device ids of
// the inner nodes in linear [x][y][z] order.
struct HetMaterials {
	const IsoAxis* tab;
	const uint8_t* ids;
};
// The heterogeneous one-pass step needs bs <= 2 and Z in {64, 128, 256, 512}.
bool het_supported(const Geo& g);
// `kname`: set to the launched instance's symbol (a static string).
// [xb0, xb1): an optional second plane range (xb0 >= x1) covered by the same
// launch (the X-slab boundary sides; two launches on the k_fused_xyz path).
// Rows longer than 512 (a multiple of 512), uniform medium, no y/z faces: the
// z-split step (k_step_tx2<..., ZS> + k_zseam); else the one-plane k_fused_xyz.
int zs_part(const Geo& g);  // lanes per part of the z-split step, 0: rows are not split
// The z split runs for these axis tables (uniform medium, floor(q) = 0): then the
// one-pass step takes rows longer than 512 with face conditions and the folded ODE.
bool zs_admissible(const Geo& g, const IsoAxis* a);
int step_free_cus(const Geo& g, int x0, int x1, int req_chunk, int cus = -1);  // cus <= 0: the device's
// Two builds of the one-pass step kernels (kernels_xyz.hip): xyz_exact keeps the
// reference's roundings (bitwise), xyz_fma contracts multiply-adds
// (gcmx_set_fp_mode).
namespace xyz_exact {
bool launch_fused_xyz(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                      int x1, hipStream_t st, int chunk = 0, const FaceBC* faces = nullptr,
                      const char** kname = nullptr, const HetMaterials* het = nullptr, int xb0 = 0,
                      int xb1 = 0);
}
namespace xyz_fma {
bool launch_fused_xyz(const double* in, double* out, const Geo& g, const IsoAxis* a, int x0,
                      int x1, hipStream_t st, int chunk = 0, const FaceBC* faces = nullptr,
                      const char** kname = nullptr, const HetMaterials* het = nullptr, int xb0 = 0,
                      int xb1 = 0);
}

}  // namespace gcmx
