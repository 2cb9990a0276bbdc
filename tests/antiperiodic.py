"""The reference's antiperiodic flux check (shared by the CPU and GPU tests).

cfemm/femmcli/test/femmcli_antiperiodicBC_flux.lua: a nonlinear (50-point
B-H steel) permanent-magnet machine sector with antiperiodic boundaries
(tests/golden/antiperiodic_flux.fem, the script's femmcli_antiperiodicBC_flux.fem),
solved, then |Bx| + |By| from mo_getpointvalues at 45 grid points
(x = -40..-20, y = -20..20, step 5 mm) compared with FEMM 4.2's values; a
point fails when |diff| > 0.02 T OR |diff| / expected > 70 %.  The script
notes the calculation "contained errors in xfemm 2.0".
"""
from __future__ import annotations

import os
import shutil

import numpy as np

from util import GOLDEN

FEM = os.path.join(GOLDEN, "antiperiodic_flux.fem")
TOL_ABS = 0.02
TOL_REL_PCT = 70.0
# B_abs_ref[0..44] of the script (FEMM42), in its x-major, y-minor order
B_ABS_REF = [
    2.0172349211547e-005, 9.980515629468256e-005, 0.0001299999163508703, 0.0001123790790807998,
    0.0001035638039144443, 4.712390174349349e-005, 1.52445645287574e-005, 2.238963159664765e-005,
    5.255076860801661e-005, 0.0001501846812706276, 0.0001875769644342095, 0.3434866174139751,
    0.3134173948888234, 0.2044994410897019, 0.007451582859305774, 0.0008821347188708024,
    6.601243412719332e-005, 7.025226578942951e-005, 0.4604507368660987, 0.7077796643063485,
    0.000977829137071488, 0.001296664349720595, 0.3067033815500693, 0.001112765134440902,
    0.001093521065145376, 0.1565090701118708, 0.2693002040535217, 0.000862706441337431,
    0.9772489557271694, 0.00123522025689945, 0.01587650688903416, 0.6762699821164218,
    0.01412679651697672, 0.002241449307702012, 0.348186232581696, 0.0007352310639869735,
    0.002163325834308883, 0.1874576095909183, 1.162091824546714, 1.0038388444812,
    0.2763546286608281, 1.001015575730773, 2.847901526518666, 0.7007337071437815,
    0.00312702704756613]
POINTS = [(x, y) for x in range(-40, -19, 5) for y in range(-20, 21, 5)]


def write_case(dst_dir) -> str:
    """The fixture meshed by oracle/mesher.py (the reference's Triangle) in dst_dir."""
    from oracle import mesher
    base = os.path.join(str(dst_dir), "antiperiodic_flux")
    shutil.copy(FEM, base + ".fem")
    mesher.write_mesh(mesher.mesh_problem(mesher.parse_geometry(FEM)), base)
    return base


def flux_post(pr, x, y, A, p, lbl):
    """oracle/pointvalues.FluxPost of a solution on the fixture's mesh (x, y in
    drawing units).  Block properties as fpproc holds them: mu_x, mu_y after
    GetSlopes(0) (fpproc.cpp:809-842: a B-H block's mu_x = B[1] / (mu0 |H[1]|)),
    H_c as read."""
    from oracle import femfile, pointvalues
    raw = femfile.parse_fem(FEM)
    props = [(b.mu_x, b.mu_y, rb.H_c) for b, rb in zip(pr.blocks, raw.blocks)]
    return pointvalues.FluxPost(x, y, A, p, lbl, [lb.BlockType for lb in raw.labels],
                                [lb.MagDir for lb in raw.labels], props, raw.LengthUnits)


def check(post):
    """The script's check(): (number failed, max |diff| T, max |diff| %, rows)."""
    failed, mx, mx_rel, rows = 0, 0.0, 0.0, []
    for (x, y), ref in zip(POINTS, B_ABS_REF):
        bx, by = post.point_b(float(x), float(y))
        v = abs(bx) + abs(by)
        diff = v - ref
        rel = 100.0 * diff / ref if ref != 0 else 0.0
        bad = abs(diff) > TOL_ABS or abs(rel) > TOL_REL_PCT
        failed += bad
        mx, mx_rel = max(mx, abs(diff)), max(mx_rel, abs(rel))
        rows.append((x, y, v, ref, rel, bad))
    return failed, mx, mx_rel, rows


def drawing_units(mesh, length_units):
    u = [2.54, 0.1, 1., 100., 0.00254, 1.e-04][length_units]   # cm per unit (FSolver::LoadMesh)
    return np.asarray(mesh.x) / u, np.asarray(mesh.y) / u
