"""The diagnostic tools stay runnable: every tools/*.py byte-compiles and every
tools/*.sh passes `bash -n` (tools/README.md)."""
import glob
import os
import py_compile
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "tools", "*.py"))),
                         ids=os.path.basename)
def test_tool_script_compiles(path, tmp_path):
    py_compile.compile(path, cfile=str(tmp_path / "x.pyc"), doraise=True)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "tools", "*.sh"))),
                         ids=os.path.basename)
def test_tool_shell_syntax(path):
    subprocess.run(["bash", "-n", path], check=True)


def test_readme_lists_every_tool():
    readme = open(os.path.join(ROOT, "tools", "README.md")).read()
    for p in glob.glob(os.path.join(ROOT, "tools", "*.py")) + glob.glob(os.path.join(ROOT, "tools", "*.sh")) \
            + glob.glob(os.path.join(ROOT, "tools", "*.hip")):
        assert os.path.basename(p) in readme, os.path.basename(p)
