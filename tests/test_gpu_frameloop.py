"""The headless frame loop (main.cpp:92-147) and its recorded-input
mode (row 3, main.cpp:155-234) end to end on the GPU: the C++ driver's last frame,
dumped as PPM, is checked against the CPU oracle (oracle/rm_oracle.c) rendering
the uniforms the reference's host step produces for that frame (RGBA8 within
1 LSB, the parity bar), and against the same frame through the Python mirror
(rmarch, byte for byte).  The test pins the driver's per-frame host step (camera
update, by-name uploads, input replay) against an independent implementation."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd", "rm_frameloop")
GOLD = os.path.join(ROOT, "tests", "golden", "input_goldens.json")

pytestmark = pytest.mark.gpu


def read_ppm(path):
    with open(path, "rb") as fh:
        data = fh.read()
    head = data.split(b"\n", 3)
    assert head[0] == b"P6" and head[2] == b"255"
    w, h = map(int, head[1].split())
    return np.frombuffer(head[3], np.uint8).reshape(h, w, 3)


def run_driver(tmp_path, *args):
    out = tmp_path / "frame.ppm"
    p = subprocess.run([DRIVER, *map(str, args), "--dump", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    return read_ppm(out), p.stdout


def render(rm, W, H, u):
    with rm.Renderer(W, H) as r:
        r.dispatch(u)
        return r.read_rgba8(flip_y=True)[..., :3]


def assert_matches_oracle(oracle, img, u, W, H):
    """The dumped PPM (top row first) against the oracle's frame (row 0 = bottom)."""
    ref = oracle.render(u, W, H, want_counts=False)["rgba8"][::-1, :, :3]
    d = np.abs(img.astype(np.int16) - ref.astype(np.int16))
    assert d.max() <= 1, f"driver frame vs oracle: max |d| {d.max()}, {(d > 1).sum()} channels over 1"


def golden_sweep_uniforms(rm, f, bounces, aa):
    """Frame f of the sweep S(120) built without librm's host code: the camera
    basis from the goldens made over the reference's vendored GLM
    (tests/golden/camera_goldens.json, case f = sweep frame f), the light of
    main.cpp:108-114, iTime = f / 60."""
    import struct
    with open(os.path.join(ROOT, "tests", "golden", "camera_goldens.json")) as fh:
        c = json.load(fh)["cases"][f]
    fl = lambda v: struct.unpack("<f", struct.pack("<I", v))[0]  # noqa: E731
    u = rm.rm_uniforms()
    for dst, key in ((u.camera.pos, "cameraPos"), (u.camera.dir, "forward"),
                     (u.camera.yAxis, "up"), (u.camera.xAxis, "right")):
        for i in range(3):
            dst[i] = fl(c[key][i])
        dst[3] = 0.0
    L = u.light
    L.position[:] = (-5.0, 5.0, -10.0)
    L.ambient[:] = (0.03, 0.04, 0.1)
    L.diffuse[:] = (0.8, 0.8, 0.8)
    L.specular[:] = (0.5, 0.5, 0.5)
    L.constant, L.linear, L.quadratic = 1.0, 0.009, 0.00032
    u.iTime = struct.unpack("<f", struct.pack("<f", f / 60.0))[0]
    u.bounceVar, u.AA, u.shadow_mode = bounces, int(aa), rm.RM_SHADOW_SOFT
    return u


def test_sweep_loop_last_frame(rm, oracle, gpu, tmp_path):
    """The driver's sweep S(120) (main.cpp:92-147 with the synthetic camera of SURVEY
    8(d)): its last frame against the oracle rendering frame 119 from the
    GLM-golden camera, so neither librm's camera nor its kernel is the reference."""
    W, H, F = 96, 64, 120
    img, log = run_driver(tmp_path, "--width", W, "--height", H, "--frames", F,
                          "--bounces", 2, "--aa", 1)
    assert f"frames {F}" in log
    u = golden_sweep_uniforms(rm, F - 1, 2, True)
    assert_matches_oracle(oracle, img, u, W, H)
    np.testing.assert_array_equal(img, render(rm, W, H, rm.sweep_uniforms(F - 1, F, 2, True, rm.RM_SHADOW_SOFT)))


@pytest.mark.parametrize("batch", [7, 32])
def test_sweep_loop_batched(rm, oracle, gpu, tmp_path, batch):
    """rm_frameloop --batch B: the same host loop, B frames per rm_dispatch_frames
    (120 = 17 x 7 + 1 and 3 x 32 + 24: a short last batch); the dumped last frame
    equals the per-frame loop's and the oracle's."""
    W, H, F = 96, 64, 120
    img, log = run_driver(tmp_path, "--width", W, "--height", H, "--frames", F,
                          "--bounces", 2, "--aa", 1, "--batch", batch)
    assert f"frames {F}" in log
    assert_matches_oracle(oracle, img, golden_sweep_uniforms(rm, F - 1, 2, True), W, H)
    np.testing.assert_array_equal(img, render(rm, W, H, rm.sweep_uniforms(F - 1, F, 2, True, rm.RM_SHADOW_SOFT)))


def script_from_golden(events):
    lines = []
    for e in events:
        if e["ev"] == "frame":
            lines.append(f"frame {_d(e['now']):.17g} {e['held'] & 15}")
        elif e["ev"] == "key":
            lines.append(f"key {e['key']} {e['action']}")
        else:
            lines.append(f"mouse {_d(e['x']):.17g} {_d(e['y']):.17g}")
    return "\n".join(lines) + "\n"


def _d(u):
    import struct
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def test_recorded_input_replay(rm, oracle, gpu, tmp_path):
    with open(GOLD) as fh:
        events = json.load(fh)["events"][:240]
    W, H = 80, 48
    script = tmp_path / "input.txt"
    script.write_text(script_from_golden(events))
    img, log = run_driver(tmp_path, "--width", W, "--height", H, "--input", script)
    nframes = sum(e["ev"] == "frame" for e in events)
    assert f"frames {nframes}" in log

    # replay the same events through the Python mirror; the driver's last frame is the
    # state after the last frame line (events after it are applied to no frame)
    last = max(i for i, e in enumerate(events) if e["ev"] == "frame")
    inp = rm.Input(W, H)
    for e in events[: last + 1]:
        if e["ev"] == "frame":
            inp.begin_frame(_d(e["now"]))
            inp.processInput(e["held"] & 15)
        elif e["ev"] == "key":
            inp.key_callback(e["key"], 0, e["action"], 0)
        else:
            inp.mouse_callback(_d(e["x"]), _d(e["y"]))
    u = inp.to_uniforms()
    assert_matches_oracle(oracle, img, u, W, H)
    np.testing.assert_array_equal(img, render(rm, W, H, u))
    # the input changed something the renderer sees
    assert (u.bounceVar, u.AA) != (0, 1) or list(u.camera.pos)[:3] != [0.0, 0.0, 0.0]


def test_escape_ends_the_loop(rm, gpu, tmp_path):
    script = tmp_path / "esc.txt"
    script.write_text("frame 0.1 0\nframe 0.2 16\nframe 0.3 0\nframe 0.4 0\n")
    _, log = run_driver(tmp_path, "--width", 32, "--height", 32, "--input", script)
    assert "frames 2" in log  # the ESC frame renders, then the window closes (main.cpp:92,157)
