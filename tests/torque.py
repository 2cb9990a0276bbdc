"""TorqueBenchmark fixtures (BASELINE configs[0]/[1]) shared by the CPU and GPU tests.

The machine is the reference's test/TorqueBenchmark.fem (byte-identical to
cfemm/femmcli/test/femmcli_antiperiodicBC_AGE_TorqueBenchmark.fem and, up to
its comment line, to femmcli_TorqueBenchmark.fem): a magnet rotor in an
air-gap element "AGE" (BdryType 6), a magnetised exterior disc joined to the
problem disc by the periodic boundaries pbc1 / pbc2 (a Kelvin-type open
boundary), one point property.  Its mesh comes from tools/gen_torque_fixtures.py
(oracle/mesher.py over the reference's Triangle); the rotor angle is the AGE's
InnerAngle, which only changes the .pbc.

The reference's own check (femmcli/test/femmcli_TorqueBenchmark.lua): the gap
torque mo_gapintegral("AGE", 0) equals the analytic sin(angle) N m, failing
when |diff| > 4.2e-5 N m OR |diff| / expected > 0.006 %.
"""
from __future__ import annotations

import os
import shutil

from util import GOLDEN

TORQUE_DIR = os.path.join(GOLDEN, "torque")
ANGLES = list(range(0, 91, 10))
# femmcli_TorqueBenchmark.lua: tq_ref (analytic), tq_tolerance, tq_toleranceRel (%)
TQ_REF = {0: 0.0, 10: 0.173648, 20: 0.342020, 30: 0.5, 40: 0.642788, 50: 0.766044,
          60: 0.866025, 70: 0.939693, 80: 0.984808, 90: 1.0}
TQ_TOL_ABS = 0.000042
TQ_TOL_REL_PCT = 0.006


def torque_ok(value: float, deg: int):
    """femmcli_TorqueBenchmark.lua check(): (ok, diff, diffRel %)."""
    exp = TQ_REF[deg]
    diff = value - exp
    rel = 100.0 * diff / exp if exp != 0 else 0.0
    return (abs(diff) <= TQ_TOL_ABS and abs(rel) <= TQ_TOL_REL_PCT), diff, rel


def _set_inner_angle(text: str, deg: float) -> str:
    """mi_modifyboundprop("AGE", 10, deg): the AGE's <innerangle>."""
    out, in_age = [], False
    for ln in text.split("\n"):
        s = ln.strip().lower()
        if s.startswith("<bdryname>"):
            in_age = '"age"' in s
        if in_age and s.startswith("<innerangle>"):
            ln = "    <innerangle> = %.17g" % deg + ("\r" if ln.endswith("\r") else "")
        out.append(ln)
    return "\n".join(out)


def write_case(dst_dir, deg: int, name: str = "TorqueBenchmark") -> str:
    """configs[0] at rotor angle ``deg``: .fem + committed mesh in ``dst_dir``;
    returns the base path (FSolver's PathName)."""
    base = os.path.join(str(dst_dir), "%s_%d" % (name, deg))
    with open(os.path.join(GOLDEN, "TorqueBenchmark.fem"), newline="") as fh:
        fem = fh.read()
    with open(base + ".fem", "w", newline="") as fh:
        fh.write(_set_inner_angle(fem, float(deg)))
    for ext in (".node", ".ele", ".edge"):
        shutil.copy(os.path.join(TORQUE_DIR, "TorqueBenchmark" + ext), base + ext)
    shutil.copy(os.path.join(TORQUE_DIR, "TorqueBenchmark_%d.pbc" % deg), base + ".pbc")
    return base


def write_fine_case(dst_dir, deg: int) -> str:
    """configs[1]: the refined (~200k-triangle) machine at rotor angle ``deg``,
    meshed now by oracle/mesher.py (needs oracle/_ref/libtriangle.so)."""
    from oracle import mesher
    base = os.path.join(str(dst_dir), "TorqueBenchmark_fine_%d" % deg)
    src = os.path.join(TORQUE_DIR, "TorqueBenchmark_fine.fem")
    with open(src, newline="") as fh:
        fem = fh.read()
    with open(base + ".fem", "w", newline="") as fh:
        fh.write(_set_inner_angle(fem, float(deg)))
    res = mesher.mesh_problem(mesher.parse_geometry(src))
    mesher.write_mesh(res, base, {"AGE": (float(deg), 0.0)})
    return base
