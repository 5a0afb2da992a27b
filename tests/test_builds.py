"""Every compile-time branch left in librm's sources is built by some test or by
the default build.  The default build is `make librm`
(__graft_entry__.build); the diagnostic builds below compile rm_kernels.hip for
gfx950 with the probes tools/ uses: RM_STATS (tools/stats_probe.py), RM_WAVE_TIMES
(tools/wave_timeline.hip) and the RM_DBL_<PHASE> cost probes (tools/ab_kernel.py
via tools/build_variant.sh), and rm_table.hip with its RM_TDBL_<PHASE> probes.
Device-only compiles: no GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

DIAG = {
    "stats+wave_times": ["-DRM_STATS=1", "-DRM_WAVE_TIMES=1"],
    "dbl_probes": ["-DRM_DBL_MARCH=1", "-DRM_DBL_BMARCH=1", "-DRM_DBL_NORMAL=1",
                   "-DRM_DBL_SHADOW=1", "-DRM_DBL_LIGHT=1", "-DRM_DBL_GAMMA=1"],
    "table_dbl_probes": ["-DRM_TDBL_MARCH=1", "-DRM_TDBL_BMARCH=1", "-DRM_TDBL_NORMAL=1",
                         "-DRM_TDBL_SHADOW=1"],
}
SOURCE = {"table_dbl_probes": "rm_table.hip"}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("name", sorted(DIAG))
def test_diagnostic_build_compiles(name, tmp_path):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "--cuda-device-only", "-c", os.path.join(CSRC, SOURCE.get(name, "rm_kernels.hip")),
           "-o", str(tmp_path / "k.o")] + DIAG[name]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
