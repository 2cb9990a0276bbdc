"""lab: the Newton AC solver single device vs row blocks on one case, with
the pass / KludgeSolve trace (XFK_TRACE_NONLINEAR=1 on stderr)."""
import copy
import os
import sys

_root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [_root, os.path.join(_root, "tests")]
os.environ["XFK_TRACE_NONLINEAR"] = "1"
from oracle import harmonic as oh  # noqa: E402
from test_gpu_harmonic_sharded import run_sharded, single  # noqa: E402
from test_gpu_newton_ac import _case, _tol  # noqa: E402
from util import CONVERGED_PRECISION, rel_err, synth_to_oracle  # noqa: E402

kind, n, nr = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
kw = _case(kind, n)
pr, mesh, kk = synth_to_oracle(kw)
Ao, st, _ = oh.solve(pr, mesh)
pr2 = copy.deepcopy(pr)
pr2.Precision = CONVERGED_PRECISION
Ac, _, _ = oh.solve(pr2, mesh)
print("oracle passes", st["newton_iters"], "tol", _tol(Ao, Ac), flush=True)
print("=== single", file=sys.stderr, flush=True)
r1, A1 = single(kk)
print("single: passes %d err %.3e" % (r1["newton_iters"], rel_err(A1, Ac)), flush=True)
for q in (1, nr):
    print("=== sharded %d" % q, file=sys.stderr, flush=True)
    out, _ = run_sharded(kk, q)
    print("sharded %d: passes %d err %.3e" % (q, out[0][0]["newton_iters"], rel_err(out[0][1], Ac)), flush=True)
