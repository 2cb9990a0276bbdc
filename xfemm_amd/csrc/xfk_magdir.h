// xfk_magdir.h -- magnetisation-direction functions of block labels (host C++).
//
// A block label's MagDirFctn is a Lua expression the reference evaluates per
// element (cfemm/fsolver/static2d.cpp:511-581, staticaxi.cpp:354-404): the
// chunk "x=..\ny=..\nr=x\nz=y\ntheta=..\nR=..\nreturn <MagDirFctn>" runs in
// the solver's Lua 4 interpreter, whose numbers are complex (the xfemm
// liblua, femmcomplex.cpp), and Re() of the returned value is the element's
// magnetisation angle in degrees.  The product evaluates the expression
// language itself -- numbers, the six centroid globals, PI, I, the math
// library, arithmetic, comparisons, and / or / not -- with the complex
// arithmetic restated operation by operation, so the angle is bit-identical
// to the reference interpreter's (tests/test_magdir.py pins it against the
// reference's own liblua compiled into oracle/_ref).  No Lua is linked into
// the product.
#pragma once

#include <memory>
#include <string>

namespace xfk {

struct MagDirExpr;   // a parsed expression (opaque)

// Parse MagDirFctn once.  Returns nullptr with `err` set to the reference's
// message (static2d.cpp:550-553) when the text is not an expression this
// evaluator accepts.
std::shared_ptr<const MagDirExpr> magdir_parse(const std::string &fctn, std::string &err);

// Evaluate for one element with nodes (x[k], y[k]) in cm (FSolver::LoadMesh
// units); `length_units` is the problem's femm::LengthUnit (the centroid is
// converted back to drawing units as static2d.cpp:521-525 does).  On success
// *t is the angle in degrees: the expression's real part, or `mag_dir` when
// the chunk returns no value (static2d.cpp:559-581).  Returns false with
// `err` set (the reference's messages) on a run-time error or a non-numeric
// result.
bool magdir_eval(const MagDirExpr &e, const double x[3], const double y[3], int length_units, double mag_dir,
                 double *t, std::string &err);

}  // namespace xfk
