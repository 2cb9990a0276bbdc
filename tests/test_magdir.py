"""Magnetisation-direction functions (MagDirFctn) -- host side, no GPU.

The product evaluates a label's Lua expression natively (xfk_magdir_eval,
xfemm_amd/csrc/xfk_magdir.cpp).  The checker is the reference's own Lua 4
interpreter (cfemm/libfemm/liblua compiled into oracle/_ref/libreflua.so,
driven as static2d.cpp:509-583 drives it).  The bar is bit-identical angles
for every element, over the reference fixture's expressions, a battery of
expressions touching every operator and math-library function, and centroids
in every length unit (negative, integral and on-axis coordinates included);
failures must carry the reference's message.
"""
import os

import numpy as np
import pytest

from oracle import femfile, oracle
from util import GOLDEN
from xfemm_amd import kernels

needs_lua = pytest.mark.skipif(not oracle.ref_lua_available(), reason="oracle/_ref/libreflua.so not built")

EXPRS = [
    # the reference fixture (test/test_lua_mag_direction.fem) and common idioms
    "theta", "theta+180", "theta-90", "-theta", "theta + 90", "90", "-45", "0.5", "-0.5",
    # arithmetic, the integer peephole (ADDI), literal negation, precedence
    "x*y", "x/y+R", "x^2+y^2", "-x^2", "2^-3*x", "- - 3 + x", "x - -3", "x-1", "x-0.5", "-0.5*x", "x-0", "-0*x",
    "1e3*x", ".5*y", "1/x", "x/(y+I)", "(x+I*y)^3", "(x+I*y)^-2", "R^0.5", "(-R)^0.5", "3-x", "(1)-x",
    # math library (radians), complex arguments, the globals PI and I
    "atan2(y,x)", "deg(atan2(y,x))+90", "sin(theta)*cos(R)", "sqrt(-R)", "abs(x)", "arg(x+I*y)*180/PI",
    "re(I*x*y)", "im(I*x)", "conj(x+I*y)", "tan(x)", "asin(0.5)", "acos(2)", "asin(x)", "acos(x/100)", "atan(I*x)",
    "atan(x)", "exp(I*x)", "log(-R)", "log10(R)", "tanh(x/10)", "tanh(-x/10)", "sinh(x/10)+cosh(y/10)",
    "min(x,y,theta)", "max(x,y,theta)", "mod(theta,45)", "floor(theta)", "ceil(theta)", "frexp(R)", "ldexp(x,3)",
    "rad(theta)", "atan2(I*y,x)", "arg(-x*y)", "arg(x-1)", "arg(conj(x)-3)", "arg(-(x*0))", "sqrt(x+I*y)",
    # comparisons and logic
    "x>0 and 90 or -90", "not (x<y) and theta or -theta", "x==x", "x~=y and 1", "(x<=y) and 3 or 4",
    "(x>=y) and 3 or 4", "r==x and z==y and 1 or 0",
    # statement forms the reference chunk allows after `return`
    "theta;", "theta, R", "theta -- a comment", "",
    # strings: numeric text, coercion in arithmetic and function arguments, concatenation
    "'45'", '"1e2"', "'30'+theta", "sin('0.5')", "x..''", "'4'..'5'", "[[12]]", "'a'<'b' and 1 or 2", "'\\0601'",
    "'2+I*3'*x", "-'7'", "'abc'", "(x..'')+1",
]

BAD = ["theta +", "foo", "foo(1)", "x(1)", "sin()", "theta end", "nil", "x < nil", "sin", "1/0*0+I*(0/0)", "''",
       "'a'+1", "x < '1'", "sin('a')", "'unfinished", "x..nil"]


def mesh_sample(n=400, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-50, 50, 3 * n)
    y = rng.uniform(-50, 50, 3 * n)
    x[:30] = np.round(x[:30])
    y[:30] = np.round(y[:30])
    x[30:60] = 0.0
    y[60:90] = 0.0
    x[90:93] = y[90:93] = 0.0
    return np.arange(3 * n).reshape(-1, 3), x, y


def evaluate(fn, *a):
    try:
        return fn(*a)
    except (ValueError, kernels.XfkError) as ex:
        return str(ex)


@needs_lua
@pytest.mark.parametrize("lu", range(6))
def test_magdir_bit_identical_to_reference_lua(lu):
    p, x, y = mesh_sample()
    for e in EXPRS:
        ref = evaluate(oracle.ref_magdir, e, p, x, y, lu, 7.0)
        got = evaluate(kernels.magdir_eval, e, p, x, y, lu, 7.0)
        if isinstance(ref, str):
            assert isinstance(got, str) and ref in got, (e, ref, got)
            continue
        assert not isinstance(got, str), (e, got)
        assert np.array_equal(ref.view(np.int64), got.view(np.int64)), (e, lu, ref[ref != got][:3], got[ref != got][:3])


@needs_lua
def test_magdir_errors_carry_the_reference_message():
    p, x, y = mesh_sample(20)
    for e in BAD:
        ref = evaluate(oracle.ref_magdir, e, p, x, y, 0, 0.0)
        got = evaluate(kernels.magdir_eval, e, p, x, y, 0, 0.0)
        assert isinstance(ref, str) and isinstance(got, str), (e, ref, got)
        assert ref in got, (e, ref, got)


def test_magdir_no_value_keeps_mag_dir():
    p, x, y = mesh_sample(5)
    t = kernels.magdir_eval("   ", p, x, y, 0, 33.0)
    assert (t == 33.0).all()


@needs_lua
def test_magdir_fixture_mesh_elements(tmp_path):
    """The reference fixture (test/test_lua_mag_direction.fem, "theta" and
    "theta+180" magnets, inches) on its own mesh: the product's directions
    equal the reference Lua's for every element of both functional labels."""
    from oracle import mesher
    src = os.path.join(GOLDEN, "test_lua_mag_direction.fem")
    base = str(tmp_path / "fx")
    mesher.write_mesh(mesher.mesh_problem(mesher.parse_geometry(src)), base)
    import shutil
    shutil.copy(src, base + ".fem")
    pr, mesh = femfile.load_problem(base)
    assert pr.LengthUnits == 0
    ref = oracle.element_magdir(pr, mesh)
    for k, lb in enumerate(pr.labels):
        sel = np.where(np.asarray(mesh.lbl) == k)[0]
        if not lb.MagDirFctn:
            assert (ref[sel] == lb.MagDir).all()
            continue
        got = kernels.magdir_eval(lb.MagDirFctn, np.asarray(mesh.p)[sel], mesh.x, mesh.y, pr.LengthUnits, lb.MagDir)
        assert len(sel) > 100
        assert np.array_equal(got.view(np.int64), ref[sel].view(np.int64)), lb.MagDirFctn


@needs_lua
@pytest.mark.parametrize("e", ['openfile("/nonexistent/xfemm/q", "r") == nil and 1 or 0', 'date() and 1 or 0'])
def test_magdir_unsupported_lua_is_named(e):
    """Valid Lua the native interpreter does not restate (files): the
    reference evaluates it, the product refuses it
    with a message naming the construct -- not a Lua error (INTEGRATION.md
    lists what is refused; tests/test_lua_interp.py covers the rest)."""
    p, x, y = mesh_sample(4)
    ref = evaluate(oracle.ref_magdir, e, p, x, y, 0, 0.0)
    assert not isinstance(ref, str), ref
    got = evaluate(kernels.magdir_eval, e, p, x, y, 0, 0.0)
    assert isinstance(got, str) and "not supported by the native Lua interpreter" in got, got
    assert "Lua error occurred" not in got
