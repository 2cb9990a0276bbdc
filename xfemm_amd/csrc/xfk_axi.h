// Axisymmetric element geometry shared by StaticAxisymmetric
// (staticaxi.cpp:215-276) and HarmonicAxisymmetric (harmonicaxi.cpp:248-330):
// the flux formulation with c0 + c1 r^2 + c2 z interpolation -- the r-weighted
// radial stiffness Mr, the axial stiffness Mz with the logarithmic mean
// radius R_hat, the diagonal fix for nodes on the axis.
#pragma once

#include <hip/hip_runtime.h>

namespace xfk {

struct AxiGeom {
    double Mx[3][3], My[3][3];   // Mr, Mz (full, symmetric)
    double R;                    // centroid radius
    double a;                    // area
    double vol;                  // 2 R a_hat
};

__device__ __forceinline__ void axi_geometry(const double (&X)[3], const double (&Y)[3], AxiGeom &G)
{
    double p[3], q[3], g[3], rn[3];
    p[0] = Y[1] - Y[2]; p[1] = Y[2] - Y[0]; p[2] = Y[0] - Y[1];
    q[0] = X[2] - X[1]; q[1] = X[0] - X[2]; q[2] = X[1] - X[0];
    g[0] = (X[2] + X[1]) / 2.; g[1] = (X[0] + X[2]) / 2.; g[2] = (X[1] + X[0]) / 2.;
    rn[0] = X[0]; rn[1] = X[1]; rn[2] = X[2];
    G.a = (p[0] * q[1] - p[1] * q[0]) / 2.;
    const double R = (X[0] + X[1] + X[2]) / 3.;
    G.R = R;
    double a_hat = 0;
    for (int j = 0; j < 3; ++j) a_hat += (rn[j] * rn[j] * p[j] / (4. * R));
    G.vol = 2. * R * a_hat;
    int flag = 0;
    for (int j = 0; j < 3; ++j) flag += (rn[j] < 1.e-06);
    double R_hat = 0.;
    if (flag == 2) {
        R_hat = R;
    } else if (flag == 1) {
        if (rn[0] < 1.e-06)
            R_hat = (fabs(rn[1] - rn[2]) < 1.e-06) ? rn[2] / 2. : (rn[1] - rn[2]) / (2. * log(rn[1]) - 2. * log(rn[2]));
        if (rn[1] < 1.e-06)
            R_hat = (fabs(rn[2] - rn[0]) < 1.e-06) ? rn[0] / 2. : (rn[2] - rn[0]) / (2. * log(rn[2]) - 2. * log(rn[0]));
        if (rn[2] < 1.e-06)
            R_hat = (fabs(rn[0] - rn[1]) < 1.e-06) ? rn[1] / 2. : (rn[0] - rn[1]) / (2. * log(rn[0]) - 2. * log(rn[1]));
    } else {
        if (fabs(q[0]) < 1.e-06)
            R_hat = (q[1] * q[1]) / (2. * (-q[1] + rn[0] * log(rn[0] / rn[2])));
        else if (fabs(q[1]) < 1.e-06)
            R_hat = (q[2] * q[2]) / (2. * (-q[2] + rn[1] * log(rn[1] / rn[0])));
        else if (fabs(q[2]) < 1.e-06)
            R_hat = (q[0] * q[0]) / (2. * (-q[0] + rn[2] * log(rn[2] / rn[1])));
        else
            R_hat = -(q[0] * q[1] * q[2]) /
                    (2. * (q[0] * rn[0] * log(rn[0]) + q[1] * rn[1] * log(rn[1]) + q[2] * rn[2] * log(rn[2])));
    }
    double K = (-1. / (2. * a_hat * R));
    for (int j = 0; j < 3; ++j)
        for (int k = j; k < 3; ++k) G.Mx[j][k] = K * p[j] * rn[j] * p[k] * rn[k];
    // something on the diagonal of axis nodes (set to zero later), for scaling
    for (int j = 0; j < 3; ++j)
        if (rn[j] < 1.e-06) G.Mx[j][j] += G.Mx[0][0] + G.Mx[1][1] + G.Mx[2][2];
    K = (-1. / (2. * a_hat * R_hat));
    for (int j = 0; j < 3; ++j)
        for (int k = j; k < 3; ++k) G.My[j][k] = K * (q[j] * rn[j]) * (q[k] * rn[k]) * (g[j] / R) * (g[k] / R);
    G.Mx[1][0] = G.Mx[0][1]; G.Mx[2][0] = G.Mx[0][2]; G.Mx[2][1] = G.Mx[1][2];
    G.My[1][0] = G.My[0][1]; G.My[2][0] = G.My[0][2]; G.My[2][1] = G.My[1][2];
}

}  // namespace xfk
