// ref_lua.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref/libreflua.so).
//
// Runs a block label's MagDirFctn through the REFERENCE's own Lua 4
// interpreter (cfemm/libfemm/liblua, compiled from /root/reference by
// oracle/Makefile, never copied) exactly as FSolver::Static2D's element loop
// does (cfemm/fsolver/static2d.cpp:509-583): centroid in CComplex, the chunk
// "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn %s", lua_dostring
// on one interpreter kept across elements (LuaInstance opens the base, string,
// math and io libraries, LuaInstance.cpp:185-197), Re of the value left on
// the stack.  The product's native evaluator (xfemm_amd/csrc/xfk_magdir.cpp)
// and the oracle's per-element directions are checked against this.
#include <cstdio>
#include <cstring>
#include <string>

#include "femmcomplex.h"
#include "lua.h"
#include "lualib.h"

#define PI 3.141592653589793238462643383   // femmconstants.h:28

// Returns 0, or -7 (Static2D's return code) with `msg` set to the reference's
// warning text.
extern "C" int ref_lua_magdir(const char *fctn, int n, const int *p, const double *x, const double *y,
                              int length_units, double mag_dir, double *t, char *msg, int msglen)
{
    double units[] = {2.54, 0.1, 1., 100., 0.00254, 1.e-04};   // static2d.cpp:67
    lua_State *lua = lua_open(4096);
    lua_baselibopen(lua);
    lua_strlibopen(lua);
    lua_mathlibopen(lua);
    lua_iolibopen(lua);
    int rc = 0;
    for (int i = 0; i < n && rc == 0; ++i) {
        const int *nd = p + 3L * i;
        char magbuff[4096];
        CComplex X;
        int j;
        for (j = 0, X = 0; j < 3; j++) X += (CComplex)(x[nd[j]] + I * y[nd[j]]);
        X = X / units[length_units] / 3.;
        snprintf(magbuff, sizeof magbuff, "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn %s", (X.re),
                 (X.im), (arg(X) * 180 / PI), (abs(X)), fctn);
        const int top1 = lua_gettop(lua);
        const int code = lua_dostring(lua, magbuff);
        t[i] = mag_dir;
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
