"""The headless frame loop (main.cpp:92-147) and its recorded-input
mode (row 3, main.cpp:155-234) end to end on the GPU: the C++ driver's last frame,
dumped as PPM, must equal the same frame rendered through the Python mirror
(rmarch) from the same uniforms.  Both paths are librm's HIP kernel; the test pins
the driver's per-frame host step (camera update, by-name uploads, input replay)."""
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


def test_sweep_loop_last_frame(rm, gpu, tmp_path):
    W, H, F = 96, 64, 4
    img, log = run_driver(tmp_path, "--width", W, "--height", H, "--frames", F,
                          "--bounces", 2, "--aa", 1)
    assert f"frames {F}" in log
    want = render(rm, W, H, rm.sweep_uniforms(F - 1, F, 2, True, rm.RM_SHADOW_SOFT))
    np.testing.assert_array_equal(img, want)


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


def test_recorded_input_replay(rm, gpu, tmp_path):
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
    np.testing.assert_array_equal(img, render(rm, W, H, u))
    # the input changed something the renderer sees
    assert (u.bounceVar, u.AA) != (0, 1) or list(u.camera.pos)[:3] != [0.0, 0.0, 0.0]


def test_escape_ends_the_loop(rm, gpu, tmp_path):
    script = tmp_path / "esc.txt"
    script.write_text("frame 0.1 0\nframe 0.2 16\nframe 0.3 0\nframe 0.4 0\n")
    _, log = run_driver(tmp_path, "--width", 32, "--height", 32, "--input", script)
    assert "frames 2" in log  # the ESC frame renders, then the window closes (main.cpp:92,157)
