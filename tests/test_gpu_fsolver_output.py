"""Where the drop-in FSolver writes its .ans (fsolver.cpp clear_old_output):
an existing large .ans is moved aside under a unique name and unlinked beside
the write, except when the path is a symlink or a hard link -- then the
reference's fopen(path, "wt") behaviour is kept: the file is truncated in
place, so the link, the target's inode and its permissions stay
(cfemm/fsolver/static2d.cpp:1038-1044 opens the .ans that way)."""
import glob
import os

import pytest

from xfemm_amd import fsolver, synth

pytestmark = pytest.mark.gpu


def _solve(base):
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.runSolver(False), fs.last_error()


def _case(tmp_path, name):
    base = str(tmp_path / name)
    synth.write_problem(base, synth.magnetostatic(150))   # .ans of ~1.5 MB (> the 1 MiB move-aside size)
    return base


def test_ans_over_an_existing_file_is_replaced_and_no_aside_file_remains(tmp_path):
    base = _case(tmp_path, "plain")
    with open(base + ".ans", "w") as fh:
        fh.write("x" * (2 << 20))
    _solve(base)
    txt = open(base + ".ans").read()
    assert "[Solution]" in txt and "x" * 64 not in txt
    assert not glob.glob(base + ".ans.xfemm-old*")


def test_symlinked_ans_is_written_through_the_link(tmp_path):
    base = _case(tmp_path, "linked")
    target = str(tmp_path / "target.ans")
    with open(target, "w") as fh:
        fh.write("x" * (2 << 20))
    os.chmod(target, 0o640)
    ino = os.stat(target).st_ino
    os.symlink(target, base + ".ans")
    _solve(base)
    assert os.path.islink(base + ".ans")
    st = os.stat(target)
    assert st.st_ino == ino and (st.st_mode & 0o777) == 0o640
    assert "[Solution]" in open(target).read()


def test_hard_linked_ans_keeps_its_inode(tmp_path):
    base = _case(tmp_path, "hard")
    other = str(tmp_path / "other.ans")
    with open(other, "w") as fh:
        fh.write("x" * (2 << 20))
    os.link(other, base + ".ans")
    _solve(base)
    assert os.stat(other).st_ino == os.stat(base + ".ans").st_ino
    assert "[Solution]" in open(other).read()
