"""Interactive input mapping: librm's rm_input_* against the
reference's GLFW globals and callbacks (main.cpp:20-39, 93-95, 155-234;
source/MousePosition.cpp:4-33; camera.cpp:16-51).

The trace in tests/golden/input_goldens.json was produced by
oracle/gen_input_goldens.cpp, which restates those callbacks with the
reference's declared types over the reference's vendored GLM 0.9.8.5, and
replays 600 pseudo-random frame / key / cursor events.  Host-only (no GPU
calls); every float is compared bit for bit."""
import ctypes as C
import json
import os
import struct

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "input_goldens.json")


def fb(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def d(u):
    return struct.unpack("<d", struct.pack("<Q", u))[0]


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as fh:
        return json.load(fh)


def snapshot(inp):
    s, cam = inp.state, inp.camera
    u = inp.to_uniforms()
    return {
        "axes": [s.zaxisPos, s.zaxisNeg, s.xaxisPos, s.xaxisNeg],
        "halfSpeed": fb(s.halfSpeed), "AA": s.AA, "showQuad": s.showQuad,
        "bounce": s.bounce, "close": s.shouldClose, "deltaTime": fb(s.deltaTime),
        "lastFrame": fb(s.lastFrame), "lastX": fb(s.lastX), "lastY": fb(s.lastY),
        "firstMouse": s.firstMouse, "yaw": fb(s.yaw), "pitch": fb(s.pitch),
        "euler": [fb(v) for v in inp.EulerAngles()],
        "cam_mouse": [fb(cam.xpos), fb(cam.ypos)],
        # what the frame uploads (main.cpp:103-106): the uniform block, not the members
        "pos": [fb(v) for v in list(u.camera.pos)[:3]],
        "dir": [fb(v) for v in list(u.camera.dir)[:3]],
        "yAxis": [fb(v) for v in list(u.camera.yAxis)[:3]],
        "xAxis": [fb(v) for v in list(u.camera.xAxis)[:3]],
    }


def test_goldens_cover_every_event_kind(gold):
    kinds = {e["ev"] for e in gold["events"]}
    assert kinds == {"frame", "key", "mouse"}
    assert "GLM 0.9.8.5" in gold["generator"]
    st = [e["state"] for e in gold["events"]]
    assert {s["bounce"] for s in st} == set(range(6))       # both clamps reached
    assert {s["AA"] for s in st} == {0, 1}
    assert any(s["close"] for s in st)                       # ESC seen
    assert {s["halfSpeed"] for s in st} == {fb(0.0), fb(1.0)}


def test_initial_state_matches_globals(rm, gold):
    inp = rm.Input(*gold["screen"])
    assert inp.AA == 1 and inp.bounce == 0 and inp.firstMouse == 1   # main.cpp:27,30,37
    assert inp.lastX == 540.0 and inp.lastY == 540.0                 # main.cpp:35-36
    assert inp.mouseSensitivity == struct.unpack("<f", struct.pack("<f", 0.001))[0]
    # the start-up camera has not run lookAt yet (main.cpp:40): compare members only
    g = gold["initial"]
    s = snapshot(inp)
    for k in ("axes", "halfSpeed", "AA", "showQuad", "bounce", "close", "deltaTime",
              "lastFrame", "lastX", "lastY", "firstMouse", "yaw", "pitch", "euler"):
        assert s[k] == g[k], k


def test_event_trace_bit_exact(rm, gold):
    inp = rm.Input(*gold["screen"])
    for i, e in enumerate(gold["events"]):
        if e["ev"] == "frame":
            inp.begin_frame(d(e["now"]))
            inp.processInput(e["held"])
        elif e["ev"] == "key":
            inp.key_callback(e["key"], 0, e["action"], 0)
        else:
            inp.mouse_callback(d(e["x"]), d(e["y"]))
        got = snapshot(inp)
        for k, v in e["state"].items():
            assert got[k] == v, f"event {i} ({e['ev']}) field {k}: {got[k]} != {v}"


def test_key_rules(rm):
    inp = rm.Input()
    for _ in range(9):
        inp.key_callback(rm.KEY_UP, 0, rm.PRESS, 0)
    assert inp.bounce == 5                                   # main.cpp:199-201
    inp.key_callback(rm.KEY_UP, 0, rm.REPEAT, 0)
    inp.key_callback(rm.KEY_DOWN, 0, rm.RELEASE, 0)
    assert inp.bounce == 5                                   # only GLFW_PRESS acts
    for _ in range(9):
        inp.key_callback(rm.KEY_DOWN, 0, rm.PRESS, 0)
    assert inp.bounce == 0                                   # main.cpp:202-204
    inp.key_callback(rm.KEY_F1, 0, rm.PRESS, 0)
    assert inp.AA == 0 and inp.to_uniforms().AA == 0         # main.cpp:206-207
    inp.key_callback(rm.KEY_L, 0, rm.PRESS, 0)
    assert inp.showQuad == 1                                 # display-only toggle


@pytest.mark.parametrize("held,half", [
    (0, 0), (1, 0), (1 | 4, 0), (2 | 8, 0),                 # none, W, W+S, A+D: full speed
    (1 | 2, 1), (1 | 8, 1), (2 | 4, 1), (4 | 8, 1), (15, 1),  # diagonals: half speed
])
def test_half_speed_rule(rm, held, half):
    inp = rm.Input()
    inp.begin_frame(0.5)
    inp.processInput(held)
    assert inp.halfSpeed == float(half)                      # main.cpp:185-193
    assert inp.camera.keyboardSpeed == (5.0 if half else 10.0)


def test_motion_moves_the_uploaded_camera(rm):
    inp = rm.Input()
    inp.begin_frame(0.0)
    inp.processInput(0)
    z0 = inp.to_uniforms().camera.pos[2]
    inp.begin_frame(0.1)
    inp.processInput(rm.HELD_W)                              # forward = -z at start-up
    z1 = inp.to_uniforms().camera.pos[2]
    assert z1 == pytest.approx(z0 - 10.0 * 0.1, abs=1e-5)
    u = inp.to_uniforms()
    assert u.iTime == pytest.approx(0.1) and u.bounceVar == 0 and u.AA == 1


def test_null_arguments_rejected(rm):
    lib = rm.lib()
    assert lib.rm_input_init(None, 10, 10) == rm.RM_ERR_INVALID
    s = rm.rm_input_state()
    assert lib.rm_input_init(C.byref(s), 0, 10) == rm.RM_ERR_INVALID
    assert lib.rm_input_key(None, rm.KEY_UP, rm.PRESS) == rm.RM_ERR_INVALID
    assert lib.rm_input_mouse(C.byref(s), 1.0, 2.0, None) == rm.RM_ERR_INVALID
