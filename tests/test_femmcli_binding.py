"""femmcli's use of FSolver through the C-ABI (include/xfemm_fsolver.h), host side.

cfemm/femmcli/LuaMagneticsCommands.cpp:817-842 (mi_analyze) creates an
FSolver, sets PathName and -- before LoadProblemFile -- previousSolutionFile
from the document (:824), then asserts the loaded solver against the document
(:830-838): ACSolver, Frequency, and the property-list sizes (equal for
boundaries, points and blocks; circuits may grow by the serial expansion;
labels exclude holes).  The reference's FEASolver::CleanUp leaves
previousSolutionFile alone (feasolver.cpp:134-172), so a preset file survives
the parse unless the .fem has its own [PrevSoln] line.  No GPU needed: these
stop before runSolver (tests/test_gpu_prev_solution.py solves through the
preset file on the device)."""
import re

import pytest

import ansfile
import torque
from oracle import femfile, oracle
from xfemm_amd import fsolver


def _doc_counts(text):
    """What the femmcli document holds: the .fem's own counts."""
    def num(tag):
        return int(re.search(r"\[%s\]\s*=\s*(\d+)" % re.escape(tag), text, re.I).group(1))
    return dict(lineproplist=num("BdryProps"), nodeproplist=num("PointProps"), blockproplist=num("BlockProps"),
                circproplist=num("CircuitProps"), labellist=num("NumBlockLabels"))


def _load(base, prev=None):
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    if prev is not None:
        fs.previousSolutionFile = prev
    ok = fs.LoadProblemFile()
    return fs, ok


def test_loaded_solver_matches_the_document(tmp_path):
    base = torque.write_case(tmp_path, 30)
    text = open(base + ".fem").read()
    doc = _doc_counts(text)
    fs, ok = _load(base)
    assert ok, fs.last_error()
    pr = femfile.parse_fem(base + ".fem")
    assert fs.ACSolver == pr.ACSolver and fs.Frequency == pr.Frequency
    got = fs.list_sizes()
    for k in ("lineproplist", "nodeproplist", "blockproplist"):
        assert got[k] == doc[k], (k, got[k], doc[k])
    assert doc["circproplist"] <= got["circproplist"]
    assert doc["labellist"] >= got["labellist"]


def _prev_case(tmp_path):
    base = torque.write_case(tmp_path, 30)
    pr, mesh = femfile.load_problem(base)
    A, _, _ = oracle.solve(pr, mesh)
    fem = open(base + ".fem").read()
    ansfile.write_static_ans(base + ".ans", fem, pr, mesh, A)
    base2 = str(tmp_path / "preset")
    with open(base2 + ".fem", "w") as fh:   # no [PrevSoln] line at all
        fh.write("\n".join(ln for ln in fem.split("\n") if not ln.strip().lower().startswith("[prevsoln]")))
    return base, base2, mesh


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
def test_preset_previous_solution_file_survives_the_parse(tmp_path):
    base, base2, mesh = _prev_case(tmp_path)
    fs, ok = _load(base2)
    assert ok and fs.NumNodes == 0                      # no previous solution: the mesh comes later
    fs, ok = _load(base2, prev=base + ".ans")
    assert ok, fs.last_error()
    assert fs.previousSolutionFile == base + ".ans"
    assert fs.NumNodes == len(mesh.x) and fs.NumEls == len(mesh.p)   # mesh taken from the .ans


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
def test_fem_prevsoln_line_overrides_the_preset(tmp_path):
    base, base2, mesh = _prev_case(tmp_path)
    with open(base2 + ".fem") as fh:
        fem = fh.read()
    with open(base2 + ".fem", "w") as fh:
        fh.write(fem.replace("[PrevType]", '[PrevSoln]    = ""\n[PrevType]', 1))
    fs, ok = _load(base2, prev=base + ".ans")
    assert ok and fs.previousSolutionFile == "" and fs.NumNodes == 0
