"""librm's glm-free Camera (rm_host.cpp) vs goldens from the reference's vendored
GLM 0.9.8.5 (tests/golden/camera_goldens.json, made by oracle/gen_camera_goldens.cpp).
Host-only: no GPU calls.  Bit-exact."""
import json
import os
import struct

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "camera_goldens.json")


def f(u):
    return struct.unpack("<f", struct.pack("<I", u))[0]


def b(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as fh:
        return json.load(fh)


def test_goldens_present(gold):
    assert len(gold["cases"]) >= 200
    assert "GLM 0.9.8.5" in gold["generator"]


def test_lookat_bit_exact(rm, gold):
    sens = f(gold["mouseSensitivity"])
    for i, c in enumerate(gold["cases"]):
        cam = rm.Camera(1080, 1080, sens, 10.0, [f(v) for v in c["pos"]], (0, 0, -1), (0, 1, 0))
        cam.setMouse(f(c["xpos"]), f(c["ypos"]))
        zN, zP, xN, xP, half = c["keys"]
        cam.lookAt(zN, zP, xN, xP, half, f(c["dt"]))
        for key, attr in (("forward", "forward"), ("up", "up"), ("right", "right"),
                          ("cameraPos", "cameraPos")):
            got = [b(v) for v in getattr(cam, attr)]
            assert got == c[key], f"case {i} {key}: {got} != {c[key]}"


def test_ctor_basis(rm, gold):
    cam = rm.Camera(1080, 1080, 0.025, 10.0, (0, 0, 0), (0, 0, -1), (0, 1, 0))
    assert [b(v) for v in cam.forward] == gold["ctor"]["forward"]
    assert [b(v) for v in cam.right] == gold["ctor"]["right"]
    # camera.cpp:13 assigns the constructor PARAMETER `up`: the member stays zero
    assert tuple(cam.up) == (0.0, 0.0, 0.0)


def test_sweep_uniforms_use_the_golden_camera(rm, gold):
    # frame f of the sweep S(120) is golden case f (pos (0,0,15), no motion)
    for fr in (0, 37, 60, 119):
        u = rm.sweep_uniforms(fr, 120, 3, True, 0)
        c = gold["cases"][fr]
        assert [b(v) for v in list(u.camera.dir)[:3]] == c["forward"]
        assert [b(v) for v in list(u.camera.yAxis)[:3]] == c["up"]
        assert [b(v) for v in list(u.camera.xAxis)[:3]] == c["right"]
        assert list(u.camera.pos) == [0.0, 0.0, 15.0, 0.0]
        assert u.camera.dir[3] == 0.0 and u.camera.xAxis[3] == 0.0  # main.cpp:103-106
        assert u.iTime == pytest.approx(fr / 60.0)


def test_default_uniforms_match_main_cpp(rm):
    u = rm.default_uniforms()
    assert list(u.light.position) == [-5.0, 5.0, -10.0]          # main.cpp:108
    assert [round(v, 6) for v in u.light.ambient] == [0.03, 0.04, 0.1]
    assert list(u.light.diffuse) == pytest.approx([0.8] * 3)
    assert list(u.light.specular) == [0.5] * 3
    assert u.light.constant == 1.0
    assert u.light.linear == pytest.approx(0.009)
    assert u.light.quadratic == pytest.approx(0.00032)
    assert u.AA == 1 and u.bounceVar == 0                       # main.cpp:27,30
    assert list(u.camera.dir)[:3] == [0.0, 0.0, -1.0]
