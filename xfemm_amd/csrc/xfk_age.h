// Air-gap elements (host side, geometry only).
//
// FSolver::Static2D and Harmonic2D add, before the triangle loop of every
// assembly, the contributions of each CAirGapElement: totalArcElements quad
// elements in the unmeshed annulus, each coupling five consecutive nodes of
// the inner ring with five of the outer ring through a 10x10 matrix that
// depends only on the geometry (static2d.cpp:191-344, harmonic2d.cpp:227-380).
// Nothing in it changes between assemblies or Newton iterations, so the host
// reduces all of it once per problem to one value per matrix entry; the GPU
// adds those values at their CSR slots after the element scatter
// (k_add_at_slots) and the entries join the CSR pattern through the same
// fill-in list as the periodic boundary conditions.
#pragma once
#include <vector>

#include "../../include/xfemm_kernels.h"

namespace xfk {

// MG of one arc element for ring shifts ci, co (already reduced as
// static2d.cpp:206-215 does) and K = dr / (R dtheta), Ki = 1 / K.
void age_matrix(double ci, double co, double K, double Ki, double MG[10][10]);

// Sum of every air-gap contribution of the problem as upper-triangle entries
// (key (r << 32) | c, r <= c), each accumulated in the reference's AddTo
// order, times `sign` (+1 Static2D; -1 Harmonic2D, whose system carries the
// opposite sign: harmonic2d.cpp:382).  Returns XFK_OK or XFK_ERR_ARG (with the
// message set) on a malformed description.
int age_entries(const xfk_problem_desc *d, double sign, std::vector<long long> &key, std::vector<double> &val);

}  // namespace xfk
