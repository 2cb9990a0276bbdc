"""Air-gap torque from a solved vector potential -- TEST INFRASTRUCTURE ONLY.

Restates the part of the reference's post-processor that its own machine test
asserts on: ``mo_gapintegral(name, 0)`` (femmcli/LuaMagneticsCommands.cpp:964),
i.e.

  * the air-gap field harmonics of every AGE   cfemm/fpproc/fpproc.cpp:1390-1610
    (A and B at the centre of each arc element from the ten-node AGE stencil,
    convolution with cos / sin of each harmonic, normalisation);
  * FPProc::gapDCTorqueIntegral                 cfemm/fpproc/fpproc.cpp:5417-5445.

The checker for BASELINE configs[0]/[1]: femmcli/test/femmcli_TorqueBenchmark.lua
expects torque = sin(rotor angle) N m on test/TorqueBenchmark.fem to
4.2e-5 N m (and femmcli_antiperiodicBC_AGE_TorqueBenchmark.lua to 0.02 N m).
"""
from __future__ import annotations

import math

import numpy as np

PI = 3.141592653589793238462643383
MUO = 1.2566370614359173e-6
LENGTH_CONV_METERS = [0.0254, 0.001, 0.01, 1.0, 2.54e-05, 1.0e-06]


def age_harmonics(age: dict, A, length_units: int = 2):
    """(nh, brc, brs, btc, bts) of one AGE (fpproc.cpp:1390-1610).

    ``age`` holds format, ri, ro, total_arc_length, inner_shift, outer_shift and
    the quadNode table qn / qw ((n+1) x 4) in the numbering of ``A``."""
    conv = LENGTH_CONV_METERS[length_units]
    ri_m, ro_m = age["ri"] * conv, age["ro"] * conv
    qn, qw = np.asarray(age["qn"]), np.asarray(age["qw"])
    n_el = qn.shape[0] - 1
    fmt = age["format"]
    R = (ri_m + ro_m) / 2.
    dr = ro_m - ri_m
    dt = (PI / 180.) * age["total_arc_length"] / float(n_el)
    if fmt == 0:
        nn = n_el // 2 + 1
        m = int(math.floor(360. / age["total_arc_length"] + 0.5))
    else:
        nn = (n_el + 1) // 2
        m = int(math.floor(180. / age["total_arc_length"] + 0.5))
    ci, co = age["inner_shift"], age["outer_shift"]
    A = np.asarray(A)
    br = np.zeros(n_el, dtype=A.dtype)
    bt = np.zeros(n_el, dtype=A.dtype)
    for k in range(n_el):
        km = n_el - 1 if k - 1 < 0 else k - 1
        kp = 1 if k + 2 > n_el else k + 2
        nnk = [qn[km, 0], qn[k, 0], qn[k, 1], qn[k + 1, 1], qn[kp, 1],
               qn[km, 2], qn[k, 2], qn[k, 3], qn[k + 1, 3], qn[kp, 3]]
        ww = [qw[km, 0], qw[k, 0], qw[k, 1], qw[k + 1, 1], qw[kp, 1],
              qw[km, 2], qw[k, 2], qw[k, 3], qw[k + 1, 3], qw[kp, 3]]
        if k == 0 and fmt == 1:
            ww[0], ww[5] = -ww[0], -ww[5]
        if k + 1 == n_el and fmt == 1:
            ww[4], ww[9] = -ww[4], -ww[9]
        a = [A[nnk[i]] * ww[i] for i in range(10)]
        br[k] = (-(ci * a[1]) - 2 * a[2] + 2 * a[3] + ci * (a[2] + a[3] - a[4])
                 - ci * ci * ci * (a[0] - 4 * a[1] + 6 * a[2] - 4 * a[3] + a[4])
                 + ci * ci * (a[0] - 5 * a[1] + 9 * a[2] - 7 * a[3] + 2 * a[4]) - 2 * a[7]
                 + 2 * a[8] + co * (-a[6] + a[7] + a[8] - a[9])
                 - co * co * co * (a[5] - 4 * a[6] + 6 * a[7] - 4 * a[8] + a[9])
                 + co * co * (a[5] - 5 * a[6] + 9 * a[7] - 7 * a[8] + 2 * a[9])) / (4 * dt * R)
        bt[k] = (ci * a[1] + 2 * a[2] + 2 * a[3] - ci * ci * (a[0] - 3 * a[1] + a[2] + 3 * a[3] - 2 * a[4])
                 + ci * (a[2] - a[3] - a[4]) + ci * ci * ci * (a[0] - 2 * a[1] + 2 * a[3] - a[4]) - co * a[6]
                 + (-2 + co) * (1 + co) * a[7] - 2 * a[8]
                 + co * (a[8] + co * (a[5] - 3 * a[6] + 3 * a[8] - 2 * a[9]) + a[9]
                         + co * co * (-a[5] + 2 * a[6] - 2 * a[8] + a[9]))) / (4 * dr)
    nh = np.zeros(nn, dtype=np.int64)
    out = np.zeros((4, nn), dtype=A.dtype)
    for j in range(nn):
        nh[j] = m * j if fmt == 0 else m * (2 * j + 1)
        s = np.zeros(4, dtype=A.dtype)
        for k in range(n_el):
            tta = (float(k) + 0.5) * dt
            tta *= nh[j]
            c, sn = math.cos(tta), math.sin(tta)
            s += (br[k] * c, br[k] * sn, bt[k] * c, bt[k] * sn)
        if nh[j] == 0 or (j == nn - 1 and fmt == 0 and n_el % 2 == 0):
            s = s / n_el
        else:
            s = s / (float(n_el) / 2.)
        out[:, j] = s
    return nh, out[0], out[1], out[2], out[3]


def gap_dc_torque(age: dict, A, depth: float, length_units: int = 2, frequency: float = 0.0) -> float:
    """FPProc::gapDCTorqueIntegral (fpproc.cpp:5417-5445); ``depth`` in length
    units as in the .fem (scaled to metres like fpproc.cpp:1612-1614)."""
    conv = LENGTH_CONV_METERS[length_units]
    depth_m = 1.0 if depth == -1 else depth * conv
    R = (age["ri"] + age["ro"]) * conv / 2.
    _, brc, brs, btc, bts = age_harmonics(age, A, length_units)
    tq = float(np.sum(np.real(brc * np.conj(btc) + brs * np.conj(bts))))
    tq *= (PI * R * R * depth_m) / MUO
    if frequency != 0:
        tq /= 2.
    return tq
