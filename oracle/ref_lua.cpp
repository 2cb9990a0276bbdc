// ref_lua.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref/libreflua.so).
//
// Runs a block label's MagDirFctn through the REFERENCE's own Lua 4
// interpreter (cfemm/libfemm/liblua, compiled from /root/reference by
// oracle/Makefile, never copied) exactly as FSolver::Static2D's element loop
// does (cfemm/fsolver/static2d.cpp:509-583): centroid in CComplex, the chunk
// "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn %s", lua_dostring
// on one interpreter kept across elements (LuaInstance opens the base, string,
// math and io libraries, then LuaInstance's own globals, LuaInstance.cpp:
// 185-208), Re of the value left on the stack.  LuaInstance.cpp itself needs
// the build-generated femmversion.h, so its five C functions are restated
// here as harness code (Complex as LuaInstance.cpp:228-241; the compatibility
// flag; femmVersion raises a Lua error; trace does nothing) and registered in
// its order, with its `pi` global -- the global table then holds the same
// names in the same order as the reference's.  The product's native evaluator (xfemm_amd/csrc/xfk_magdir.cpp)
// and the oracle's per-element directions are checked against this.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "femmcomplex.h"
#include "lua.h"
#include "lualib.h"

#define PI 3.141592653589793238462643383   // femmconstants.h:28

static bool compat_mode = false;

static int h_complex(lua_State *L)   // LuaInstance::luaComplex (LuaInstance.cpp:228-241)
{
    CComplex y;
    int numArgs = lua_gettop(L);
    if (numArgs == 2) y = lua_tonumber(L, 1) + I * lua_tonumber(L, 2);
    else if (numArgs == 1) y = lua_tonumber(L, 1);
    else y = 0;
    lua_pushnumber(L, y);
    return 1;
}
static int h_setcompat(lua_State *L)
{
    if (lua_gettop(L) != 0) compat_mode = (1 == lua_tonumber(L, 1).Re());
    return 0;
}
static int h_getcompat(lua_State *L)
{
    lua_pushnumber(L, CComplex(compat_mode ? 1.0 : 0.0));
    return 1;
}
static int h_femmversion(lua_State *L)
{
    lua_error(L, "femmVersion: not available in this harness");
    return 0;
}
static int h_trace(lua_State *) { return 0; }

// One interpreter for the whole element loop, as the reference keeps one per
// FSolver: element i runs its label's function (`fctn_of(i)`, NULL: the
// label's MagDir, nothing run).  Axisymmetric problems use staticaxi.cpp's
// chunk (r and z first, staticaxi.cpp:366-367).  Returns 0, or -7 (Static2D's
// return code) with `msg` set to the reference's warning text.
template <class F>
static int run_elements(F fctn_of, const double *mag_dirs_of_elem, int n, const int *p, const double *x,
                        const double *y, int length_units, int axisymmetric, double *t, char *msg, int msglen)
{
    double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};   // static2d.cpp:67
    srand(1);   // the C library's generator as a fresh fsolver process has it (random())
    lua_State *lua = lua_open(4096);
    lua_baselibopen(lua);
    lua_strlibopen(lua);
    lua_mathlibopen(lua);
    lua_iolibopen(lua);
    compat_mode = false;
    lua_register(lua, "Complex", h_complex);   // LuaInstance.cpp:200-207
    lua_register(lua, "setcompatibilitymode", h_setcompat);
    lua_register(lua, "getcompatibilitymode", h_getcompat);
    lua_register(lua, "femmVersion", h_femmversion);
    lua_register(lua, "trace", h_trace);
    lua_pushnumber(lua, CComplex(PI));
    lua_setglobal(lua, "pi");
    int rc = 0;
    for (int i = 0; i < n && rc == 0; ++i) {
        const char *fctn = fctn_of(i);
        t[i] = mag_dirs_of_elem[i];
        if (!fctn) continue;
        const int *nd = p + 3L * i;
        char magbuff[4096];
        CComplex X;
        int j;
        for (j = 0, X = 0; j < 3; j++) X += (CComplex)(x[nd[j]] + I * y[nd[j]]);
        X = X / units[length_units] / 3.;
        snprintf(magbuff, sizeof magbuff,
                 axisymmetric ? "r=%.17g\nz=%.17g\nx=r\ny=z\ntheta=%.17g\nR=%.17g\nreturn %s"
                              : "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn %s",
                 (X.re), (X.im), (arg(X) * 180 / PI), (abs(X)), fctn);
        const int top1 = lua_gettop(lua);
        const int code = lua_dostring(lua, magbuff);
        if (code != 0) {
            snprintf(msg, msglen, "Lua error occurred when evaluating:\n\"%s\"", fctn);
            rc = -7;
            break;
        }
        const int top2 = lua_gettop(lua);
        if (top2 != top1) {
            const char *s = lua_tostring(lua, -1);
            if (s == nullptr || s[0] == '\0') {   // (the reference builds a std::string from it)
                snprintf(msg, msglen, "\"%s\" does not evaluate to a numerical value", fctn);
                rc = -7;
                break;
            }
            t[i] = Re(lua_tonumber(lua, -1));
            lua_pop(lua, 1);   // as the reference: one value popped (unsafe mode)
        }
    }
    lua_close(lua);
    return rc;
}

// One function over n elements (a planar label's elements).
extern "C" int ref_lua_magdir(const char *fctn, int n, const int *p, const double *x, const double *y,
                              int length_units, double mag_dir, double *t, char *msg, int msglen)
{
    std::vector<double> md((size_t)n, mag_dir);
    return run_elements([&](int) { return fctn; }, md.data(), n, p, x, y, length_units, 0, t, msg, msglen);
}

// A whole problem's element loop: label lbl[i]'s function (NULL or "" for
// none) and MagDir.
extern "C" int ref_lua_magdir_labels(const char *const *fctns, const double *mag_dirs, int n, const int *p,
                                     const int *lbl, const double *x, const double *y, int length_units,
                                     int axisymmetric, double *t, char *msg, int msglen)
{
    std::vector<double> md((size_t)n);
    for (int i = 0; i < n; ++i) md[i] = mag_dirs[lbl[i]];
    return run_elements([&](int i) -> const char * {
        const char *f = fctns[lbl[i]];
        return (f && *f) ? f : nullptr;
    }, md.data(), n, p, x, y, length_units, axisymmetric, t, msg, msglen);
}
