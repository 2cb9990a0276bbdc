// xfk_magdir.cpp -- MagDirFctn per element (see xfk_magdir.h) over the native
// Lua 4 interpreter (xfk_lua.cpp), and the host-only C-ABI xfk_magdir_eval.
//
// What is restated (temudschin/xfemm @ 2025-02-04): the element loop's Lua
// handling of static2d.cpp:509-583 / staticaxi.cpp:350-406 -- the centroid X
// (the CComplex sum of the three nodes / units[LengthUnits] / 3), the chunk,
// the error and non-numeric messages, Re(lua_tonumber) of the text
// lua_tostring left, and the label's MagDir when nothing is returned.
#include "xfk_magdir.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

namespace xfk {
namespace {

std::string quoted(const char *fmt, const std::string &fctn)
{
    std::vector<char> buf(fctn.size() + 128);
    std::snprintf(buf.data(), buf.size(), fmt, fctn.c_str());
    return std::string(buf.data());
}

std::string unsupported(const std::string &fctn, const std::string &what)
{
    return "MagDirFctn \"" + fctn + "\": " + what +
           " not supported by the native Lua interpreter (the reference's Lua would evaluate it)";
}

}  // namespace

bool MagDir::eval(const std::string &fctn, const double x[3], const double y[3], int length_units, double mag_dir,
                  double *t, std::string &err)
{
    static const double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};   // femm::LengthUnit in cm
    // X = sum (x + I y) / units / 3 (static2d.cpp:521-525), CComplex operation by operation
    lua::Cx X{0., 0.};
    for (int j = 0; j < 3; ++j) {
        const lua::Cx node{x[j] + 0.0 * y[j], 1.0 * y[j]};   // x + I*y
        X = {X.re + node.re, X.im + node.im};
    }
    X = {X.re / units[length_units], X.im / units[length_units]};
    X = {X.re / 3., X.im / 3.};
    lua::ElementResult r;
    try {
        r = S_.run_element(fctn, X);
    } catch (const lua::Unsupported &u) {
        err = unsupported(fctn, u.what());
        return false;
    }
    if (r.error) {   // LUA_ERRRUN / LUA_ERRSYNTAX (static2d.cpp:539-556)
        err = quoted("Lua error occurred when evaluating:\n\"%s\"", fctn);
        return false;
    }
    if (r.nresults == 0) {   // nothing returned: the label's MagDir stays
        *t = mag_dir;
        return true;
    }
    // lua_tostring, then lua_tonumber of that text (static2d.cpp:563-577)
    if (!r.text || r.str.empty()) {
        err = quoted("\"%s\" does not evaluate to a numerical value", fctn);
        return false;
    }
    lua::Cx v{0., 0.};   // lua_tonumber of a text luaO_str2d rejects is 0
    if (!lua::text_to_number(r.str.c_str(), &v)) v = lua::Cx{0., 0.};
    *t = v.re;
    return true;
}

bool MagDir::repeatable(std::string &err) const
{
    if (S_.state_changed()) {
        err = unsupported("(any)",
                          "a chunk that changes Lua state (globals, tables that outlive their element, the "
                          "compatibility mode) in a nonlinear problem, whose every Newton pass re-runs the chunks,");
        return false;
    }
    if (S_.leaked() > 0) {
        err = unsupported("(any)",
                          "a chunk returning several values in a nonlinear problem (the reference leaves the extra "
                          "values on its Lua stack in every Newton pass until it overflows)");
        return false;
    }
    return true;
}

void set_error(const std::string &msg);   // xfk_api.hip

}  // namespace xfk

extern "C" int xfk_magdir_eval(const char *fctn, int n_elems, const int *p, const double *x, const double *y,
                               int length_units, double mag_dir, double *t)
{
    if (!fctn || n_elems < 0 || (n_elems > 0 && (!p || !x || !y || !t)) || length_units < 0 || length_units > 5) {
        xfk::set_error("xfk_magdir_eval: bad arguments");
        return -1;   // XFK_ERR_ARG
    }
    xfk::MagDir md(false);
    std::string err;
    for (int i = 0; i < n_elems; ++i) {
        const double X[3] = {x[p[3LL * i]], x[p[3LL * i + 1]], x[p[3LL * i + 2]]};
        const double Y[3] = {y[p[3LL * i]], y[p[3LL * i + 1]], y[p[3LL * i + 2]]};
        if (!md.eval(fctn, X, Y, length_units, mag_dir, t + i, err)) {
            xfk::set_error(err);
            return -1;
        }
    }
    return 0;
}

extern "C" int xfk_magdir_eval_labels(int n_labels, const char *const *fctns, const double *mag_dirs, int n_elems,
                                      const int *p, const int *lbl, const double *x, const double *y,
                                      int length_units, int axisymmetric, int repeats, double *t)
{
    if (n_labels < 0 || n_elems < 0 || (n_labels > 0 && (!fctns || !mag_dirs)) ||
        (n_elems > 0 && (!p || !lbl || !x || !y || !t)) || length_units < 0 || length_units > 5) {
        xfk::set_error("xfk_magdir_eval_labels: bad arguments");
        return -1;
    }
    for (int i = 0; i < n_elems; ++i)
        if (lbl[i] < 0 || lbl[i] >= n_labels) {
            xfk::set_error("xfk_magdir_eval_labels: label index out of range");
            return -1;
        }
    xfk::MagDir md(axisymmetric != 0);
    std::string err;
    bool any = false;
    for (int i = 0; i < n_elems; ++i) {
        const char *f = fctns[lbl[i]];
        if (!f || !*f) {
            t[i] = mag_dirs[lbl[i]];
            continue;
        }
        const double X[3] = {x[p[3LL * i]], x[p[3LL * i + 1]], x[p[3LL * i + 2]]};
        const double Y[3] = {y[p[3LL * i]], y[p[3LL * i + 1]], y[p[3LL * i + 2]]};
        if (!md.eval(f, X, Y, length_units, mag_dirs[lbl[i]], t + i, err)) {
            xfk::set_error(err);
            return -1;
        }
        any = true;
    }
    if (any && repeats && !md.repeatable(err)) {
        xfk::set_error(err);
        return -1;
    }
    return 0;
}

extern "C" int xfk_lua_run(const char *chunk, char *out, long long cap, long long *out_len)
{
    if (!chunk || cap < 0 || (cap > 0 && !out)) {
        xfk::set_error("xfk_lua_run: bad arguments");
        return -1;
    }
    xfk::lua::Session S(false);
    std::string text;
    int status;
    try {
        status = S.run_chunk(chunk, &text);
    } catch (const xfk::lua::Unsupported &u) {
        xfk::set_error(std::string(u.what()) + " not supported by the native Lua interpreter");
        return -1;
    }
    if (out_len) *out_len = (long long)text.size();
    if (cap > 0) {
        const size_t n = std::min<size_t>((size_t)cap - 1, text.size());
        std::memcpy(out, text.data(), n);
        out[n] = '\0';
    }
    if (status != 0) {
        xfk::set_error(status == 3 ? "Lua syntax error" : "Lua run-time error");
        return -2;
    }
    return 0;
}
