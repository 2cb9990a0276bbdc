// xfk_magdir.h -- magnetisation-direction functions of block labels (host C++).
//
// A block label's MagDirFctn is Lua the reference runs per element
// (cfemm/fsolver/static2d.cpp:511-581, staticaxi.cpp:354-404): the chunk
// "x=..\ny=..\nr=x\nz=y\ntheta=..\nR=..\nreturn <MagDirFctn>" through
// lua_dostring on the solver's one Lua 4 interpreter, whose numbers are
// complex (the xfemm liblua, femmcomplex.cpp); Re() of the last returned value
// is the element's magnetisation angle in degrees.  The product runs it on
// xfk_lua.cpp, a native restatement of that interpreter (language, tables,
// base / string / math libraries, LuaInstance's additions), one state per
// problem, every element in assembly order -- so the angle is bit-identical to
// the reference's (tests/test_magdir.py pins it against the reference's own
// liblua compiled into oracle/_ref).  No Lua is linked into the product.
#pragma once

#include <string>

#include "xfk_lua.h"

namespace xfk {

class MagDir {
public:
    // one interpreter for a problem's element loop (axisymmetric: the chunk
    // of staticaxi.cpp, which sets r and z before x and y)
    explicit MagDir(bool axisymmetric) : S_(axisymmetric) {}

    // One element with nodes (x[k], y[k]) in cm (FSolver::LoadMesh units);
    // `length_units` is the problem's femm::LengthUnit (the centroid goes back
    // to drawing units as static2d.cpp:521-525 does).  On success *t is the
    // angle in degrees: the chunk's last value's real part, or `mag_dir` when
    // it returns none (static2d.cpp:559-581).  Returns false with `err` set:
    // the reference's messages for a Lua error or a non-numeric result, or a
    // "not supported by the native Lua interpreter" message for what xfk_lua.h
    // lists as refused.
    bool eval(const std::string &fctn, const double x[3], const double y[3], int length_units, double mag_dir,
              double *t, std::string &err);

    // After the last element of a problem whose Newton loop runs the element
    // loop again every pass (a nonlinear problem): false (with `err`) when
    // the chunks changed state a later pass would see, or left values on the
    // reference's stack that accumulate pass after pass.
    bool repeatable(std::string &err) const;

private:
    lua::Session S_;
};

}  // namespace xfk
