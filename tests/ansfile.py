"""Test infrastructure: a WriteStatic2D-layout .ans (static2d.cpp:1038-1195)
from an oracle answer, to serve as a [PrevSoln] on the CPU (the GPU tests use
the .ans FSolver writes)."""
import numpy as np

UNITCONV = [2.54, 0.1, 1., 100., 0.00254, 1.e-04]


def write_static_ans(path, fem_text, pr, mesh, A):
    cf = UNITCONV[pr.LengthUnits]
    out = [fem_text.rstrip("\n"), "[Solution]", "%i" % len(mesh.x)]
    for i in range(len(mesh.x)):
        out.append("%s\t%s\t%s\t%i" % (_g(mesh.x[i] / cf), _g(mesh.y[i] / cf), _g(A[i]), mesh.marker[i]))
    out.append("%i" % len(mesh.lbl))
    for i in range(len(mesh.lbl)):
        out.append("%i\t%i\t%i\t%i" % (mesh.p[i, 0], mesh.p[i, 1], mesh.p[i, 2], mesh.lbl[i]))
    out.append("%i" % len(pr.labels))
    out += ["1\t0"] * len(pr.labels)
    out.append("%i" % len(mesh.pbc))
    out += ["%i\t%i\t%i" % tuple(r) for r in mesh.pbc]
    out.append("%i" % len(mesh.ages))
    for a in mesh.ages:
        out.append('"%s"' % a.get("name", "AGE"))
        out.append("%i %s %s %s %s %s %s %s %i %s %s" % (
            a["format"], _g(a.get("inner_angle", 0.0)), _g(a.get("outer_angle", 0.0)), _g(a["ri"]), _g(a["ro"]),
            _g(a["total_arc_length"]), _g(0.0), _g(0.0), len(a["qn"]) - 1, _g(a["inner_shift"]),
            _g(a["outer_shift"])))
        for qn, qw in zip(np.asarray(a["qn"]), np.asarray(a["qw"])):
            out.append("%i %s %i %s %i %s %i %s" % (qn[0], _g(qw[0]), qn[1], _g(qw[1]), qn[2], _g(qw[2]), qn[3],
                                                     _g(qw[3])))
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")


def _g(v):
    return "%.17g" % v


def with_prev(fem_text, prev_path, prev_type):
    """The .fem text with [PrevSoln] / [PrevType] set."""
    out = []
    for ln in fem_text.split("\n"):
        s = ln.strip().lower()
        if s.startswith("[prevsoln]"):
            ln = '[PrevSoln]    = "%s"' % prev_path
        elif s.startswith("[prevtype]"):
            ln = "[PrevType]    =  %d" % prev_type
        out.append(ln)
    return "\n".join(out)
