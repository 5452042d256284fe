// launch.hpp -- host-side launchers exported by the kernel translation units.
#pragma once

#include "common.hpp"

namespace gcmx {

// kernels_generic.hip
bool launch_stage_generic(const double* cur, double* nxt, const Geo& g, int s,
                          const AxisTable* tabs, const uint8_t* mat, hipStream_t st);
void launch_fill_random(double* cur, const Geo& g, const int gstart[3], long long GY,
                        long long GZ, uint64_t seed, hipStream_t st);
void launch_copy_box(double* dst, const Geo& gd, const double* src, const Geo& gs,
                     const int dmin[3], const int smin[3], const int ext[3], hipStream_t st);
void launch_border_fill(double* cur, const Geo& g, int axis, int inner_sign, int n_nodes,
                        const int* nodes_d, int n_q, const int* qs_d, const double* vals_d,
                        hipStream_t st);

// kernels_fast.hip -- 3-D, homogeneous, isotropic-elastic zero pattern.
// `tab` points to the device AxisTable of material 0 for the stage's axis.
// x range [x0, x1) of planes to update (slab scheduling); each returns false
// when no compiled variant covers the configuration.
bool iso_pattern_fits(int s, const double* U, const double* U1, const double* L);
bool launch_march(const double* cur, double* nxt, const Geo& g, int s, const AxisTable* tab,
                  int x0, int x1, hipStream_t st);
bool launch_line_z(const double* cur, double* nxt, const Geo& g, const AxisTable* tab, int x0,
                   int x1, hipStream_t st);
bool launch_fused_yz(const double* in, double* out, const Geo& g, const AxisTable* ty,
                     const AxisTable* tz, int x0, int x1, hipStream_t st);
bool fused_yz_supported(const Geo& g);

}  // namespace gcmx
