"""The largest frames rm_create accepts (1..65536 per side, rm_api.hip rm_create), against the oracle.

Reference: shaders/computeShader.glsl:291-344 per pixel; main.cpp:123 dispatches
one invocation per pixel of the window's texture (texture.cpp:19), whose size the
reference never bounds.  The production kernels index the image with 64-bit
offsets; a 65536 x 65536 frame has 2^32 pixels, so any 32-bit offset would wrap
in its upper half.  These tests check:
  * the widest and the tallest frames on every pixel (one row / one column of
    tiles, the grid at its largest x or y extent);
  * 65536 x 65536 frames of both kernels (16 GiB of RGBA8, rendered into a torch
    buffer through rm_set_output_rgba8) on rows at both ends and around the 2^31
    and 2^32 pixel offsets, against the oracle's rows.
Bar: RGBA8 within 1 LSB.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _threads() -> int:
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(period))))
    except (OSError, ValueError):
        pass
    return n


def _close(img, ref):
    d = np.abs(img.astype(np.int16) - ref.astype(np.int16))
    assert d.max() <= 1, (int(d.max()), int((d.max(-1) > 1).sum()))


@pytest.mark.parametrize("W,H", [(65536, 40), (40, 65536)], ids=["max-width", "max-height"])
@pytest.mark.parametrize("aa", [True, False], ids=["k_sample", "k_pixel"])
def test_extreme_aspect_whole_frame(rm, oracle, gpu, W, H, aa):
    u = rm.sweep_uniforms(61, 120, 3 if aa else 1, aa, rm.RM_SHADOW_SOFT)
    with rm.Renderer(W, H) as r:
        r.dispatch(u)
        img = r.read_rgba8()
    ref = oracle.render(u, W, H, nthreads=_threads(), want_counts=False)
    _close(img, ref["rgba8"])


@pytest.mark.parametrize("aa", [True, False], ids=["k_sample", "k_pixel"])
def test_max_frame_rows_past_2_pow_32_pixels(rm, oracle, gpu, aa):
    import torch
    W = H = 65536
    u = rm.sweep_uniforms(30, 120, 3 if aa else 0, aa, rm.RM_SHADOW_SOFT if aa else rm.RM_SHADOW_HARD)
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")  # 16 GiB
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8) as r:
        r.set_output_rgba8(out.data_ptr())
        r.dispatch(u)
        r.synchronize()
        r.set_output_rgba8(None)
    # rows 32767 / 32768 straddle pixel offset 2^31, the last rows end at 2^32
    rows = [0, 1, 32767, 32768, 49151, 65534, 65535]
    img = out[rows].cpu().numpy()
    del out
    torch.cuda.empty_cache()
    ref = oracle.render(u, W, H, rows=rows, nthreads=_threads(), want_counts=False)
    _close(img, ref["rgba8"])
    assert (img[..., 3] == 255).all()  # every pixel of these rows was written
