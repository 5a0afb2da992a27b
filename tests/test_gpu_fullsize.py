"""The production kernels at BASELINE.json's full sizes, against the CPU oracle.

Reference: shaders/computeShader.glsl:291-344 (one pixel, 1 or 4 samples),
dispatched per frame by main.cpp:92-147.  The renderers here are created with
counters off, so they run the kernels bench.py times (k_sample<false> /
k_pixel<false>, every early exit taken), not the counting build.  The oracle
renders a row sample of the same frames (all of them would take minutes on the
host); the bars are the parity bars of tests/test_gpu_parity.py: RGBA8 within
1 LSB, RGBA32F within 2e-6 with the same NaN mask.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows(H, n, seed):
    """Fixed rows (bottom, top, the middle band where the horizon and the longest
    marches are) plus a seeded random sample."""
    fixed = {0, 1, H // 4, H // 2 - 1, H // 2, H // 2 + 1, H // 2 + H // 20, 3 * H // 4, H - 1}
    rng = np.random.default_rng(seed)
    extra = set(int(x) for x in rng.choice(H, size=n, replace=False))
    return sorted(fixed | extra)


def _compare(img8, img32, rows, ref):
    d = np.abs(img8[rows].astype(np.int16) - ref["rgba8"].astype(np.int16))
    assert d.max() <= 1, f"RGBA8 max |delta| {d.max()}, {(d.max(-1) > 1).sum()} pixels over 1"
    a, b = img32[rows], ref["rgba32f"]
    na, nb = np.isnan(a), np.isnan(b)
    np.testing.assert_array_equal(na, nb)
    ok = ~na
    assert np.abs(a[ok] - b[ok]).max() <= 2e-6


@pytest.mark.parametrize("cfg", [(3840, 2160, 3, [0, 61, 119]), (3840, 2160, 5, [30, 90])],
                         ids=["cfg3-4K-b3", "cfg4-4K-b5"])
def test_production_kernel_full_size_vs_oracle(rm, oracle, gpu, cfg):
    W, H, b, frames = cfg
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F) as r:
        for f in frames:
            u = rm.sweep_uniforms(f, 120, b, True, rm.RM_SHADOW_SOFT)
            r.dispatch(u)
            img8, img32 = r.read_rgba8(), r.read_rgba32f()
            rows = _rows(H, 40, seed=f)
            ref = oracle.render(u, W, H, rows=rows, want_counts=False)
            _compare(img8, img32, rows, ref)


def test_cfg5_graph_replay_8k_vs_dispatch_and_oracle(rm, oracle, gpu):
    """BASELINE cfg 5: 7680x4320, 3 bounces, 4x supersampling, animated sweep
    replayed from the captured hipGraph (rm_graph_dispatch).  Every frame equals a
    plain rm_dispatch render byte for byte and an oracle row sample within the
    parity bars."""
    W, H = 7680, 4320
    frames = [0, 37, 74, 119]
    outs = rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F
    with rm.Renderer(W, H, outputs=outs) as g, rm.Renderer(W, H, outputs=outs) as p:
        g.graph_enable(True)
        for f in frames:
            u = rm.sweep_uniforms(f, 120, 3, True, rm.RM_SHADOW_SOFT)
            g.graph_dispatch(u)
            p.dispatch(u)
            g8, p8 = g.read_rgba8(), p.read_rgba8()
            np.testing.assert_array_equal(g8, p8)
            g32 = g.read_rgba32f()
            np.testing.assert_array_equal(g32.view(np.uint32), p.read_rgba32f().view(np.uint32))
            rows = _rows(H, 24, seed=1000 + f)
            ref = oracle.render(u, W, H, rows=rows, want_counts=False)
            _compare(g8, g32, rows, ref)
