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


def test_profile_summaries_use_the_profiling_settings():
    """tools/summarize_all.sh summarises each configuration of tools/profile_all.sh with the
    same PMC settings (kind, config, steps, frames per launch): a batched configuration's
    counters are divided by its frames per launch, so a mismatch would misstate the per-frame
    VALU and HBM figures that bench.py's roofline reads from profiles/."""
    import re
    prof = open(os.path.join(ROOT, "tools", "profile_all.sh")).read()
    summ = open(os.path.join(ROOT, "tools", "summarize_all.sh")).read()
    ran = {m.group(5): (m.group(1), m.group(2), m.group(3), m.group(4)) for m in re.finditer(
        r"PROF_KIND=(\S+) PROF_CFG=(\d+) PROF_STEPS=(\d+) PROF_BATCH=(\d+) bash tools/profile_round.sh "
        r"\$R\"_(\w+)\"", prof)}
    summed = {m.group(5): (m.group(1), m.group(2), m.group(3), m.group(4)) for m in re.finditer(
        r"^run (\S+) (\d+) (\d+) (\d+) \"\$\{SRC\}_(\w+)\"", summ, re.M)}
    assert ran and ran == summed, (ran, summed)
