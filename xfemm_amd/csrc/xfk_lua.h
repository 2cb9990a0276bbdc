// xfk_lua.h -- the Lua 4.0 interpreter of FSolver's magnetisation-direction
// functions, restated natively (host C++, no Lua linked).
//
// The reference runs a block label's MagDirFctn as the chunk
//   "x=%.17g\ny=%.17g\nr=x\nz=y\ntheta=%.17g\nR=%.17g\nreturn <MagDirFctn>"
// (static2d.cpp:530-531; staticaxi.cpp:366-367 sets r and z first) through
// lua_dostring on ONE interpreter per FSolver (fsolver.cpp:85, LuaInstance.cpp
// :185-208: the base, string, math and io libraries, Complex, pi, ...), for
// every element in assembly order, leaving the results on the stack and
// popping one (LuaInstance::LuaStackMode::Unsafe).  This interpreter restates
// that: Lua 4.0's language (lparser.cpp, lvm.cpp, ldo.cpp) with the xfemm
// complex number (femmcomplex.cpp) and tag methods (ltm.cpp), Lua 4.0's
// tables as the chained scatter table of ltable.cpp (so traversal order --
// next, foreach, `for k, v in t` -- is the reference's for number and string
// keys), the base library
// (lbaselib.cpp), the string library with its pattern matcher (lstrlib.cpp),
// the math library (lmathlib.cpp) and LuaInstance's Complex / pi /
// compatibility-mode functions.  Globals persist from element to element as
// they do in the reference.
//
// What is refused (an Unsupported exception naming the construct -- never a
// silent difference): the io library but write() on the standard handles
// (dofile of a text file runs), gcinfo, femmVersion (a build-generated constant), call's
// error-method argument, an error caught by call / dostring while
// _ERRORMESSAGE or _ALERT is not the library's, recursion deeper than 200
// calls, more than 3000 values left on the reference's 4096-slot stack (it
// overflows near there), more than 10^9 steps, 5 * 10^7 live objects or 10^5
// dostring chunks for one element, nesting beyond 1000 levels or pattern
// recursion beyond 5000 (the reference's limits there: its C stack, memory).  random / randomseed run
// glibc's rand() restated, seeded as a fresh reference process has it.
// Addresses (tostring of a table / function, table keys that are tables or
// functions, whose traversal order follows their address in the reference)
// are this process's, not the reference's.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>

namespace xfk {
namespace lua {

struct Cx {
    double re, im;
};

// valid Lua this interpreter does not restate (see above)
class Unsupported : public std::runtime_error {
public:
    explicit Unsupported(const std::string &what) : std::runtime_error(what) {}
};

struct Interp;

// luaO_str2d (lobject.cpp:138-147): a number's text as the reference reads it
// back (lua_tonumber of the string static2d.cpp:577 leaves)
bool text_to_number(const char *s, Cx *out);

// What lua_dostring of one element's chunk left for static2d.cpp:537-581.
struct ElementResult {
    bool error = false;       // lua_dostring returned non-zero (syntax or run-time error)
    int nresults = 0;         // values the chunk returned (left on the stack)
    bool text = false;        // lua_tostring(lua, -1) is not NULL (a number or a string)
    std::string str;          // ... and its text
};

class Session {
public:
    explicit Session(bool axisymmetric);
    ~Session();
    Session(const Session &) = delete;
    Session &operator=(const Session &) = delete;

    // One element: the chunk's prelude for the centroid X (drawing units,
    // static2d.cpp:521-525) and "return <fctn>", truncated to the reference's
    // 4096-byte buffer.  Throws Unsupported.
    ElementResult run_element(const std::string &fctn, Cx X);

    // true once a chunk wrote a global other than the prelude's six, wrote
    // into a table that outlived its element, or changed the compatibility
    // mode: a second pass over the elements (a Newton pass) could then give
    // other angles
    bool state_changed() const;
    // values left on the reference's stack so far (all but the popped one)
    long long leaked() const;

    // A whole chunk, as lua_dostring on this interpreter (a femmcli script):
    // 0, or the Lua error status (1 run-time, 3 syntax).  `output` (if not
    // null) receives what print / write send to the standard output.
    // Throws Unsupported.
    int run_chunk(const std::string &text, std::string *output);

private:
    std::unique_ptr<Interp> I;
};

}  // namespace lua
}  // namespace xfk
