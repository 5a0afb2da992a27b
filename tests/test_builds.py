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


BUILD = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd", "build")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
# Scratch bytes per lane each production kernel may use: none for the built-in
# kernels; the generic table kernel's batch kernels (every production frame since
# round 6, a single one as a batch of one) none in the 5-slot instances, 8 B in
# some 8-slot ones (round 6: the fast plane's centre and normal moved from scalar
# registers to LDS took the reference-shaped kernel's last spill; round 5: the output index
# re-formed after the march and the expiries' first values formed where each march
# starts; round 4: 28-32 B, and 588 B once after a change to its bounce loop).
# The single-frame table kernels are counting kernels only (k_table_*<true, KL>).
# (keys: substrings of the mangled names -- k_pixel<false>, k_sample<false>, the
# batched k_*_frames and the table batch kernels k_table_*_frames<KL, SL>)
SCRATCH_MAX = {"7k_pixelILb0E": 0, "8k_sampleILb0E": 0, "14k_pixel_frames": 0,
               "15k_sample_frames": 0, "20k_table_pixel_framesILi5E": 0, "21k_table_sample_framesILi5E": 0,
               "20k_table_pixel_frames": 8, "21k_table_sample_frames": 8}


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not installed")
@pytest.mark.parametrize("obj", ["rm_kernels.o", "rm_kernels_aa.o", "rm_table.o"])
def test_production_kernels_scratch(obj, tmp_path):
    """The in-tree build's gfx950 code objects (make librm, __graft_entry__.build):
    the private segment of every production kernel, from its kernel descriptor."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_scene_table import _kernel_private_sizes
    src = os.path.join(BUILD, obj)
    if not os.path.exists(src):
        pytest.skip("librm not built")
    shutil.copy(src, tmp_path / "x.o")
    subprocess.run([OBJDUMP, "--offloading", "x.o"], cwd=tmp_path, capture_output=True, check=True)
    cos = [p for p in os.listdir(tmp_path) if "gfx950" in p]
    assert len(cos) == 1, os.listdir(tmp_path)
    priv = _kernel_private_sizes(open(tmp_path / cos[0], "rb").read())
    if obj == "rm_table.o":  # production frames are batches (of one): no single-frame production kernels
        assert not any("k_table_sampleILb0E" in k or "k_table_pixelILb0E" in k for k in priv), priv
    seen = 0
    for sym, size in priv.items():
        for key, cap in SCRATCH_MAX.items():
            if key in sym:
                seen += 1
                assert size <= cap, (sym, size, cap)
    assert seen > 0, priv
