"""GPU tests of the C-ABI contract (include/rm_api.h): uniform setters with the
reference's by-name semantics (shader.hpp:19-69), error behaviour, readback
orientation, device interop, timing, row sharding; plus full-size property
tests at BASELINE sizes (4K cfg 3 / cfg 4) where the oracle would be too slow."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def render(rm, u, W, H, **kw):
    with rm.Renderer(W, H, **kw) as r:
        r.dispatch(u)
        return r.read_rgba8()


def test_setters_by_name_equal_struct_upload(rm, gpu):
    """main.cpp:99-120 sets every uniform by name each frame; that must equal
    uploading the same values as one struct."""
    W, H = 96, 64
    u = rm.sweep_uniforms(25, 120, 2, True, 0)
    ref = render(rm, u, W, H)
    with rm.Renderer(W, H) as r:
        assert r.setFloat("iTime", u.iTime) == 0
        wg = 39
        assert r.setuInt("workgroups", wg) == 0
        for nm in ("pos", "dir", "yAxis", "xAxis"):
            assert r.setVec4(f"camera.{nm}", *list(getattr(u.camera, nm))) == 0
        for nm in ("position", "ambient", "diffuse", "specular"):
            assert r.setVec3(f"light.{nm}", *list(getattr(u.light, nm))) == 0
        assert r.setFloat("light.constant", u.light.constant) == 0
        assert r.setFloat("light.linear", u.light.linear) == 0
        assert r.setFloat("light.quadratic", u.light.quadratic) == 0
        assert r.setBool("AA", True) == 0
        assert r.setInt("bounceVar", 2) == 0
        assert r.setFloat("drand48", 0.123) == 0          # accepted, unused (glsl:61)
        assert r.setVec3("mouse", 0.1, 0.2, 0.3) == 0     # accepted, unused (glsl:63)
        assert r.setVec2("iMouse", 4.0, 5.0) == 0         # accepted, unused (glsl:64)
        r.dispatch()
        got = r.read_rgba8()
    np.testing.assert_array_equal(got, ref)


def test_unknown_uniform_is_a_visible_noop(rm, gpu):
    """GL location -1: glUniform is a silent no-op; librm returns
    RM_WARN_UNKNOWN_UNIFORM and changes nothing."""
    with rm.Renderer(32, 32) as r:
        before = bytes(r.get_uniforms())
        assert r.setFloat("no_such_uniform", 3.0) == rm.RM_WARN_UNKNOWN_UNIFORM
        assert r.setVec3("light.colour", 1, 2, 3) == rm.RM_WARN_UNKNOWN_UNIFORM
        assert bytes(r.get_uniforms()) == before


def test_setter_type_and_range_errors(rm, gpu):
    with rm.Renderer(32, 32) as r:
        with pytest.raises(rm.RMError):
            r.setVec3("iTime", 1, 2, 3)          # wrong component count
        with pytest.raises(rm.RMError):
            r.setInt("bounceVar", 6)             # main.cpp:199-204 caps at 5
        with pytest.raises(rm.RMError):
            r.setInt("iTime", 1)                 # float uniform
        assert r.get_uniforms().bounceVar == 0   # unchanged after the errors


def test_readback_before_dispatch_is_an_error(rm, gpu):
    with rm.Renderer(16, 16) as r:
        with pytest.raises(rm.RMError) as e:
            r.read_rgba8()
        assert e.value.code == rm.RM_ERR_STATE


def test_disabled_format_is_an_error(rm, gpu):
    with rm.Renderer(16, 16, outputs=rm.RM_OUT_RGBA8) as r:
        r.dispatch(rm.sweep_uniforms(0))
        with pytest.raises(rm.RMError):
            r.read_rgba32f()
        with pytest.raises(rm.RMError):
            r.counters()


def test_flip_y_puts_the_top_row_first(rm, gpu):
    u = rm.sweep_uniforms(10, 120, 1, False, 0)
    with rm.Renderer(40, 30, outputs=3) as r:
        r.dispatch(u)
        a = r.read_rgba8()
        b = r.read_rgba8(flip_y=True)
        fa = r.read_rgba32f(flip_y=True)
    np.testing.assert_array_equal(a[::-1], b)
    np.testing.assert_array_equal(rm.quantize_rgba8(fa), b)
    # row 0 is the bottom of the screen (quad.hpp:9): the floor is at the bottom
    assert a[0].mean() != a[-1].mean()


def test_pitched_readback(rm, gpu):
    W, H = 33, 7
    with rm.Renderer(W, H) as r:
        r.dispatch(rm.sweep_uniforms(3))
        tight = r.read_rgba8()
        buf = np.zeros((H, W * 4 + 12), np.uint8)
        rc = rm.lib().rm_read_rgba8(r.handle, buf.ctypes.data, W * 4 + 12, 0)
        assert rc == 0
    np.testing.assert_array_equal(buf[:, : W * 4].reshape(H, W, 4), tight)
    assert (buf[:, W * 4:] == 0).all()


def test_external_output_and_stream_interop(rm, gpu):
    import torch
    W, H = 64, 48
    u = rm.sweep_uniforms(50, 120, 3, True, 0)
    ref = render(rm, u, W, H)
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    with rm.Renderer(W, H) as r:
        r.set_stream(s.cuda_stream)
        r.set_output_rgba8(out.data_ptr())
        assert r.output_rgba8_ptr() == out.data_ptr()
        r.dispatch(u)
        s.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        np.testing.assert_array_equal(r.read_rgba8(), ref)  # reads the external image
        r.set_output_rgba8(None)
        r.set_stream(None)


def test_kernel_timing(rm, gpu):
    with rm.Renderer(128, 128) as r:
        r.enable_timing(True)
        for f in range(3):
            r.dispatch(rm.sweep_uniforms(f))
        ms, n = r.kernel_time_ms(reset=True)
        assert n == 3 and ms > 0
        ms, n = r.kernel_time_ms()
        assert n == 0


@pytest.mark.parametrize("aa", [True, False], ids=["k_sample", "k_pixel"])
@pytest.mark.parametrize("N,R,R0", [(2, 8, 8), (3, 4, 4), (8, 8, 8), (2, 8, 7), (4, 8, 5), (8, 8, 7),
                                    (3, 4, 9)])
@pytest.mark.parametrize("W", [80, 83])  # 16-B row copies / per-pixel copies in k_unshard
@pytest.mark.parametrize("fmt", ["rgba8", "rgb8"])
def test_shards_assemble_to_the_full_frame(rm, gpu, aa, N, R, R0, W, fmt):
    """Virtual ranks of the (weighted) interleave: every shard
    rendered into its slot of one gather buffer and assembled by k_unshard equals
    the full render byte for byte; also with packed RGB shards (API version 6,
    rm_config.shard_format: 3 B per pixel, alpha 255 restored by the un-shard)."""
    import torch
    H = 61
    k = rm.RM_KERNEL_PIXEL
    u = rm.sweep_uniforms(70, 120, 3, aa, 0)
    full = render(rm, u, W, H, kernel=k)
    cap = rm.shard_rows_cap(H, R, N, R0)
    bpp = 3 if fmt == "rgb8" else 4
    sf = rm.RM_SHARD_RGB8 if fmt == "rgb8" else rm.RM_SHARD_RGBA8
    gathered = torch.zeros((N, cap, W, bpp), dtype=torch.uint8, device="cuda")
    frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    rs = [rm.Renderer(W, H, kernel=k, row_block=R, shard=i, nshards=N, rank0_rows=R0, shard_format=sf)
          for i in range(N)]
    for i, r in enumerate(rs):
        r.set_output_rgba8(gathered[i].data_ptr())
        r.dispatch(u)
        r.synchronize()
    rs[0].unshard_rgba8(gathered.data_ptr(), frame.data_ptr())
    rs[0].synchronize()
    np.testing.assert_array_equal(frame.cpu().numpy(), full)
    for r in rs:
        r.close()


@pytest.mark.parametrize("aa", [True, False], ids=["k_sample", "k_pixel"])
def test_rgb8_shard_is_the_rgba8_shard_without_alpha(rm, gpu, aa):
    """An RGB8 shard image (rm_config.shard_format, API version 6) holds exactly the
    R, G, B bytes of the RGBA8 shard, packed; its readback (rm_read_rgba8) expands
    it with alpha 255, which is every real pixel's alpha (the reference's constant
    1.0); a bad shard_format is refused."""
    import torch
    W, H, N, R, R0 = 37, 29, 3, 4, 3
    u = rm.sweep_uniforms(55, 120, 2, aa, 0)
    for s in range(N):
        rows = rm.shard_global_rows(H, R, s, N, R0)
        real = rows >= 0
        with rm.Renderer(W, H, row_block=R, shard=s, nshards=N, rank0_rows=R0,
                         shard_format=rm.RM_SHARD_RGBA8) as a, \
             rm.Renderer(W, H, row_block=R, shard=s, nshards=N, rank0_rows=R0,
                         shard_format=rm.RM_SHARD_RGB8) as b:
            a.dispatch(u)
            b.dispatch(u)
            ia, ib = a.read_rgba8(), b.read_rgba8()
            np.testing.assert_array_equal(ib[real], ia[real])
            assert (ia[real][..., 3] == 255).all() and (ib[..., 3] == 255).all()
            # the device bytes: packed rows of 3 x width
            dev = torch.zeros(len(rows) * W * 3, dtype=torch.uint8, device="cuda")
            b.set_output_rgba8(dev.data_ptr())
            b.dispatch(u)
            b.synchronize()
            packed = dev.cpu().numpy().reshape(len(rows), W, 3)
            np.testing.assert_array_equal(packed[real], ia[real][..., :3])
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(W, H, row_block=R, shard=0, nshards=N, shard_format=7)
    assert e.value.code == rm.RM_ERR_INVALID


# ---- full-size properties (oracle too slow at these sizes) ----------------------------
@pytest.mark.parametrize("cfg", [(3840, 2160, 3, 7), (3840, 2160, 5, 90)])
def test_full_size_kernels_agree_and_are_deterministic(rm, gpu, cfg):
    W, H, b, f = cfg
    u = rm.sweep_uniforms(f, 120, b, True, 0)
    with rm.Renderer(W, H, outputs=3, kernel=rm.RM_KERNEL_PIXEL) as r:
        r.dispatch(u)
        a32 = r.read_rgba32f()
        r.dispatch(u)
        a32b = r.read_rgba32f()
    # an independent implementation of the same scene: the reference scene as a
    # runtime table through the generic k_table_* kernels (no scene-specific proofs)
    with rm.Renderer(W, H, outputs=3) as r:
        r.set_scene(rm.default_scene())
        r.dispatch(u)
        w32 = r.read_rgba32f()
        w8 = r.read_rgba8()
    np.testing.assert_array_equal(a32, a32b)          # idempotent dispatch
    np.testing.assert_array_equal(a32, w32)           # built-in == table kernel
    np.testing.assert_array_equal(w8, rm.quantize_rgba8(w32))
    assert np.isfinite(a32).all() and (a32[..., 3] == 1.0).all()


def test_full_size_counters_match_between_kernels(rm, gpu):
    W, H = 3840, 2160
    u = rm.sweep_uniforms(44, 120, 3, True, 0)
    cs = []
    for table in (False, True):  # built-in scene kernel / the same scene as a table
        with rm.Renderer(W, H, counters=True) as r:
            if table:
                r.set_scene(rm.default_scene())
            r.dispatch(u)
            cs.append((r.counters(), r.sdf_counts()))
    assert cs[0][0] == cs[1][0]
    np.testing.assert_array_equal(cs[0][1], cs[1][1])
    assert cs[0][0]["rays"] == W * H * 4
    assert int(cs[0][1].sum(dtype=np.uint64)) == cs[0][0]["sdf_evals"]


def test_full_size_rows_match_oracle_sample(rm, oracle, gpu):
    """A sparse row sample of a full 4K cfg-3 frame against the oracle."""
    W, H = 3840, 2160
    u = rm.sweep_uniforms(100, 120, 3, True, 0)
    with rm.Renderer(W, H, counters=True) as r:
        r.dispatch(u)
        img = r.read_rgba8()
        sc = r.sdf_counts()
    rows = [0, 1, 700, 1079, 1080, 1085, 1300, 2159]
    ref = oracle.render(u, W, H, rows=rows)
    np.testing.assert_array_equal(sc[rows], ref["sdf_counts"])
    assert np.abs(img[rows].astype(int) - ref["rgba8"].astype(int)).max() <= 1


def test_graph_replay_matches_dispatch(rm, gpu):
    """hipGraph frame replay (cfg 5 path): an animated sweep replayed from two
    captured graphs equals plain dispatches frame for frame, including an AA
    toggle (re-capture) and an external output buffer."""
    import torch
    W, H = 160, 90
    frames = [(f, b, aa) for f, b, aa in [(0, 3, True), (1, 3, True), (2, 3, True), (3, 1, False),
                                          (4, 1, False), (5, 3, True)]]
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    with rm.Renderer(W, H, outputs=3) as g, rm.Renderer(W, H, outputs=3) as r:
        g.graph_enable(True)
        for f, b, aa in frames:
            u = rm.sweep_uniforms(f, 120, b, aa, 0)
            r.dispatch(u)
            g.graph_dispatch(u)
            np.testing.assert_array_equal(g.read_rgba32f(), r.read_rgba32f())
        g.set_output_rgba8(out.data_ptr())
        u = rm.sweep_uniforms(9, 120, 3, True, 0)
        g.graph_dispatch(u)
        g.synchronize()
        r.dispatch(u)
        np.testing.assert_array_equal(out.cpu().numpy(), r.read_rgba8())
        g.enable_timing(True)
        for f in range(4):
            g.graph_dispatch(rm.sweep_uniforms(f, 120, 3, True, 0))
        ms, n = g.kernel_time_ms(reset=True)
        assert n == 4 and ms > 0


def test_graph_refuses_counters(rm, gpu):
    with rm.Renderer(32, 32, counters=True) as r:
        with pytest.raises(rm.RMError):
            r.graph_enable(True)


def test_graph_back_to_back_frames_keep_their_constants(rm, gpu):
    """Frames replayed back to back without host syncs, each into its own
    output buffer: the per-frame constants set on the graph's kernel node must
    not leak into a launch still in flight."""
    import torch
    W, H, n = 320, 180, 6
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(n)]
    us = [rm.sweep_uniforms(10 * f, 120, 3, True, 0) for f in range(n)]
    with rm.Renderer(W, H) as g:
        g.graph_enable(True)
        for f in range(n):
            g.set_output_rgba8(outs[f].data_ptr())
            g.graph_dispatch(us[f])
        g.synchronize()
    with rm.Renderer(W, H) as r:
        for f in range(n):
            r.dispatch(us[f])
            np.testing.assert_array_equal(outs[f].cpu().numpy(), r.read_rgba8(), err_msg=f"frame {f}")


def test_unshard_with_offset_pointers(rm, gpu):
    """rm_unshard_rgba8 takes caller device pointers: 4-byte-offset (not 16-B
    aligned) shard and frame buffers take the per-pixel copy path."""
    import torch
    W, H, N, R = 80, 45, 3, 4
    u = rm.sweep_uniforms(20, 120, 1, False, 0)
    full = render(rm, u, W, H)
    cap = rm.shard_rows_cap(H, R, N)
    gbuf = torch.zeros(N * cap * W * 4 + 16, dtype=torch.uint8, device="cuda")
    fbuf = torch.zeros(H * W * 4 + 16, dtype=torch.uint8, device="cuda")
    g0, f0 = gbuf.data_ptr() + 4, fbuf.data_ptr() + 4
    rs = [rm.Renderer(W, H, row_block=R, shard=i, nshards=N) for i in range(N)]
    for i, r in enumerate(rs):
        r.set_output_rgba8(g0 + i * cap * W * 4)
        r.dispatch(u)
        r.synchronize()
    rs[0].unshard_rgba8(g0, f0)
    rs[0].synchronize()
    got = fbuf[4:4 + H * W * 4].cpu().numpy().reshape(H, W, 4)
    np.testing.assert_array_equal(got, full)
    for r in rs:
        r.close()
