"""rmarch — Python host mirror of the reference's host API over librm's C-ABI.

The reference (Qirias/OpenGL-RayMarching-in-Compute-Shader) drives its compute
shader from C++: a ``Camera`` (source/camera.{hpp,cpp}), a ``Texture``
(source/texture.{hpp,cpp}), and the program/uniform helpers of
source/shader.hpp (``CreateCompute``, ``useShader``, ``setFloat`` ...), then
``glDispatchCompute`` + ``glMemoryBarrier`` (main.cpp:99-125).  This module
exposes the same names with the same argument meaning on top of librm
(include/rm_api.h).  The C++ mirror of the same surface is include/rm/*.hpp.

librm has no CPU backend: every render goes through the HIP kernels, and a
missing ``librm.so`` or a missing GPU raises instead of falling back.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBRM_PATH = os.environ.get("RM_LIBRM", os.path.join(_PKG_DIR, "librm.so"))

# ---- status codes / enums (include/rm_api.h) ---------------------------------
RM_OK = 0
RM_WARN_UNKNOWN_UNIFORM = 1
RM_ERR_INVALID = -1
RM_ERR_HIP = -2
RM_ERR_NOMEM = -3
RM_ERR_NO_DEVICE = -4
RM_ERR_STATE = -5
RM_ERR_COMM = -6

RM_API_VERSION = 6
RM_CONFIG_MAGIC = 0x36434D52

RM_MAX_BATCH = 32
RM_OUT_RGBA8 = 1
RM_OUT_RGBA32F = 2
RM_SHADOW_SOFT = 0
RM_SHADOW_HARD = 1
RM_KERNEL_AUTO = 0
RM_KERNEL_PIXEL = 1
RM_SHARD_AUTO = 0   # RGB8 shards once the context gathers, RGBA8 otherwise (rm_config.shard_format)
RM_SHARD_RGBA8 = 1
RM_SHARD_RGB8 = 2


class RMError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"librm error {code}: {msg}")
        self.code = code


# ---- POD structs (must match include/rm_api.h exactly) -----------------------
class rm_camera(C.Structure):
    _fields_ = [("pos", C.c_float * 4), ("dir", C.c_float * 4),
                ("yAxis", C.c_float * 4), ("xAxis", C.c_float * 4)]


class rm_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("ambient", C.c_float * 3),
                ("diffuse", C.c_float * 3), ("specular", C.c_float * 3),
                ("constant", C.c_float), ("linear", C.c_float), ("quadratic", C.c_float)]


class rm_uniforms(C.Structure):
    _fields_ = [("camera", rm_camera), ("light", rm_light), ("iTime", C.c_float),
                ("bounceVar", C.c_int32), ("AA", C.c_int32), ("workgroups", C.c_uint32),
                ("drand48", C.c_float), ("mouse", C.c_float * 3), ("iMouse", C.c_float * 2),
                ("shadow_mode", C.c_int32)]


class rm_counters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("march_steps", C.c_uint64),
                ("reflect_steps", C.c_uint64), ("shadow_steps", C.c_uint64),
                ("normals", C.c_uint64), ("lights", C.c_uint64), ("sdf_evals", C.c_uint64)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class rm_config(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("magic", C.c_uint32), ("width", C.c_int32), ("height", C.c_int32), ("device", C.c_int32),
                ("outputs", C.c_int32), ("kernel", C.c_int32), ("counters", C.c_int32),
                ("row_block", C.c_int32), ("shard", C.c_int32), ("nshards", C.c_int32),
                ("rank0_rows", C.c_int32), ("shard_format", C.c_int32), ("ngpus", C.c_int32),
                ("devices", C.POINTER(C.c_int32))]


class rm_camera_state(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("angleY", C.c_float),
                ("angleX", C.c_float), ("mouseSensitivity", C.c_float),
                ("keyboardSpeed", C.c_float), ("xpos", C.c_float), ("ypos", C.c_float),
                ("cameraPos", C.c_float * 3), ("forward", C.c_float * 3),
                ("up", C.c_float * 3), ("right", C.c_float * 3)]


class rm_input_state(C.Structure):
    _fields_ = [("zaxisPos", C.c_int32), ("zaxisNeg", C.c_int32), ("xaxisPos", C.c_int32),
                ("xaxisNeg", C.c_int32), ("AA", C.c_int32), ("showQuad", C.c_int32),
                ("halfSpeed", C.c_float), ("bounce", C.c_int32), ("deltaTime", C.c_float),
                ("lastFrame", C.c_float), ("lastX", C.c_float), ("lastY", C.c_float),
                ("firstMouse", C.c_int32), ("pitch", C.c_float), ("yaw", C.c_float),
                ("mouseSensitivity", C.c_float), ("shouldClose", C.c_int32)]


class rm_primitive(C.Structure):
    _fields_ = [("type", C.c_int32), ("swizzle", C.c_int32), ("id", C.c_int32),
                ("paint", C.c_int32), ("material", C.c_float), ("color", C.c_float * 3),
                ("center", C.c_float * 3), ("param", C.c_float * 7)]


# runtime scene table (include/rm_api.h)
RM_MAX_PRIMITIVES = 32
PRIM_SPHERE, PRIM_BOX, PRIM_BLEND, PRIM_TORUS, PRIM_CAPSULE, PRIM_PLANE = range(6)
SWIZZLE_XYZ, SWIZZLE_XZY = 0, 1
PAINT_SOLID, PAINT_CHECKERS = 0, 1
REFLECTIVE, MATTE = 1.0, 0.0


def primitive(type: int, center=(0.0, 0.0, 0.0), param=(), color=(1.0, 1.0, 1.0), id: int = 0,
              material: float = REFLECTIVE, swizzle: int = SWIZZLE_XYZ,
              paint: int = PAINT_SOLID) -> rm_primitive:
    """One scene-table entry (a RayHit-producing primitive, glsl:83-121)."""
    p = rm_primitive(type=type, swizzle=swizzle, id=id, paint=paint, material=material)
    p.color[:] = list(color)
    p.center[:] = list(center)
    p.param[:] = list(param) + [0.0] * (7 - len(param))
    return p


def default_scene() -> list:
    """The reference's scene (glsl:107-123) as table entries."""
    n = C.c_int32(0)
    out = (rm_primitive * RM_MAX_PRIMITIVES)()
    _check(lib().rm_default_scene(out, RM_MAX_PRIMITIVES, C.byref(n)))
    return [out[i] for i in range(n.value)]


def scene_words(prims: Sequence[rm_primitive]) -> np.ndarray:
    """The table as rm_set_scene compiles it for the device (rm_scene_compile; host only):
    uint32 words, the entries then the exit header (csrc/rm_internal.hpp)."""
    n = len(prims)
    tbl = (rm_primitive * max(n, 1))(*prims)
    nw = C.c_size_t(0)
    _check(lib().rm_scene_compile(tbl, n, None, 0, C.byref(nw)))
    out = (C.c_uint32 * nw.value)()
    _check(lib().rm_scene_compile(tbl, n, out, nw.value, C.byref(nw)))
    return np.frombuffer(out, np.uint32).copy()


# GLFW key / action codes (glfw3.h) and held-key bits, as in include/rm_api.h
KEY_A, KEY_D, KEY_L, KEY_S, KEY_W = 65, 68, 76, 83, 87
KEY_ESCAPE, KEY_DOWN, KEY_UP, KEY_F1 = 256, 264, 265, 290
RELEASE, PRESS, REPEAT = 0, 1, 2
HELD_W, HELD_A, HELD_S, HELD_D, HELD_ESCAPE = 1, 2, 4, 8, 16


# ---- library loading --------------------------------------------------------------
_lib: Optional[C.CDLL] = None

_P = C.c_void_p
_SIGS = {
    "rm_api_version": (C.c_int, []),
    "rm_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rm_config_init": (C.c_int, [C.POINTER(rm_config), C.c_int32, C.c_int32]),
    "rm_create": (C.c_int, [C.POINTER(_P), C.POINTER(rm_config)]),
    "rm_destroy": (None, [_P]),
    "rm_last_error": (C.c_char_p, [_P]),
    "rm_set_bool": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "rm_set_int": (C.c_int, [_P, C.c_char_p, C.c_int32]),
    "rm_set_uint": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_uint32)]),
    "rm_set_float": (C.c_int, [_P, C.c_char_p, C.c_float]),
    "rm_set_vec2": (C.c_int, [_P, C.c_char_p, C.c_float, C.c_float]),
    "rm_set_vec3": (C.c_int, [_P, C.c_char_p, C.c_float, C.c_float, C.c_float]),
    "rm_set_vec4": (C.c_int, [_P, C.c_char_p, C.c_float, C.c_float, C.c_float, C.c_float]),
    "rm_set_uniforms": (C.c_int, [_P, C.POINTER(rm_uniforms)]),
    "rm_get_uniforms": (C.c_int, [_P, C.POINTER(rm_uniforms)]),
    "rm_default_uniforms": (C.c_int, [C.POINTER(rm_uniforms)]),
    "rm_dispatch": (C.c_int, [_P]),
    "rm_dispatch_frames": (C.c_int, [_P, C.POINTER(rm_uniforms), C.c_int32]),
    "rm_read_frame_rgba8": (C.c_int, [_P, C.c_int32, _P, C.c_size_t, C.c_int]),
    "rm_read_frame_rgba32f": (C.c_int, [_P, C.c_int32, _P, C.c_size_t, C.c_int]),
    "rm_synchronize": (C.c_int, [_P]),
    "rm_read_rgba8": (C.c_int, [_P, _P, C.c_size_t, C.c_int]),
    "rm_read_rgba32f": (C.c_int, [_P, _P, C.c_size_t, C.c_int]),
    "rm_get_counters": (C.c_int, [_P, C.POINTER(rm_counters)]),
    "rm_read_sdf_counts": (C.c_int, [_P, _P]),
    "rm_graph_enable": (C.c_int, [_P, C.c_int]),
    "rm_graph_dispatch": (C.c_int, [_P]),
    "rm_set_stream": (C.c_int, [_P, _P]),
    "rm_set_output_rgba8": (C.c_int, [_P, _P]),
    "rm_get_output_rgba8": (C.c_int, [_P, C.POINTER(_P)]),
    "rm_wait_output": (C.c_int, [_P, _P]),
    "rm_unshard_rgba8": (C.c_int, [_P, _P, _P]),
    "rm_unshard_batch_rgba8": (C.c_int, [_P, _P, C.c_int32, C.c_int32, _P]),
    "rm_enable_timing": (C.c_int, [_P, C.c_int]),
    "rm_kernel_time_ms": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_int]),
    "rm_frame_phases": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double)]),
    "rm_shard_rows": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rm_shard_to_global": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rm_shard_owner": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rm_camera_init": (C.c_int, [C.POINTER(rm_camera_state), C.c_int32, C.c_int32, C.c_float,
                                 C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                 C.POINTER(C.c_float)]),
    "rm_camera_set_mouse": (C.c_int, [C.POINTER(rm_camera_state), C.c_float, C.c_float]),
    "rm_camera_look_at": (C.c_int, [C.POINTER(rm_camera_state), C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_float]),
    "rm_camera_to_uniform": (C.c_int, [C.POINTER(rm_camera_state), C.POINTER(rm_camera)]),
    "rm_input_init": (C.c_int, [C.POINTER(rm_input_state), C.c_int32, C.c_int32]),
    "rm_input_begin_frame": (C.c_int, [C.POINTER(rm_input_state), C.c_double]),
    "rm_input_process": (C.c_int, [C.POINTER(rm_input_state), C.c_uint32,
                                   C.POINTER(rm_camera_state)]),
    "rm_input_key": (C.c_int, [C.POINTER(rm_input_state), C.c_int32, C.c_int32]),
    "rm_input_mouse": (C.c_int, [C.POINTER(rm_input_state), C.c_double, C.c_double,
                                 C.POINTER(rm_camera_state)]),
    "rm_input_euler_angles": (C.c_int, [C.POINTER(rm_input_state), C.POINTER(C.c_float)]),
    "rm_input_to_uniforms": (C.c_int, [C.POINTER(rm_input_state), C.POINTER(rm_camera_state),
                                       C.POINTER(rm_uniforms)]),
    "rm_default_scene": (C.c_int, [C.POINTER(rm_primitive), C.c_int32, C.POINTER(C.c_int32)]),
    "rm_set_scene": (C.c_int, [_P, C.POINTER(rm_primitive), C.c_int32]),
    "rm_get_scene": (C.c_int, [_P, C.POINTER(rm_primitive), C.c_int32, C.POINTER(C.c_int32)]),
    "rm_scene_specialize": (C.c_int, [_P, C.c_int]),
    "rm_scene_kernel_waves": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "rm_scene_compile": (C.c_int, [C.POINTER(rm_primitive), C.c_int32, C.POINTER(C.c_uint32),
                                   C.c_size_t, C.POINTER(C.c_size_t)]),
    "rm_jit_code_object": (C.c_int, [C.POINTER(rm_primitive), C.c_int32, C.c_char_p, C.c_void_p,
                                     C.c_size_t, C.POINTER(C.c_size_t)]),
    "rm_sweep_uniforms": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.POINTER(rm_uniforms)]),
    "rm_comm_unique_id": (C.c_int, [C.c_void_p, C.c_size_t]),
    "rm_comm_init": (C.c_int, [_P, C.c_void_p, C.c_int32, C.c_int32]),
    "rm_comm_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                               C.POINTER(C.c_int32)]),
    "rm_comm_rccl_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rm_comm_set_timeout": (C.c_int, [_P, C.c_int32]),
    "rm_comm_check": (C.c_int, [_P]),
}
COMM_ID_BYTES = 128
EXPORTED_SYMBOLS = tuple(_SIGS)


def lib() -> C.CDLL:
    """Load librm.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIBRM_PATH):
            raise RuntimeError(
                f"librm.so not found at {LIBRM_PATH}: build it with `make librm` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        # PyTorch-ROCm bundles its own libamdhip64.so.7.  Load it first so that
        # librm binds to the same HIP runtime (same SONAME) and device
        # pointers / streams / RCCL buffers are shared with torch; loading
        # librm first would bring /opt/rocm's copy in as a second runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIBRM_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int, ctx=None) -> int:
    if rc < 0:
        msg = lib().rm_last_error(ctx)
        raise RMError(rc, msg.decode() if msg else "")
    return rc


def device_count() -> int:
    n = C.c_int(0)
    lib().rm_device_count(C.byref(n))
    return n.value


# ---- uniforms ------------------------------------------------------------------------
def default_uniforms() -> rm_uniforms:
    u = rm_uniforms()
    _check(lib().rm_default_uniforms(C.byref(u)))
    return u


def sweep_uniforms(frame: int, nframes: int = 120, bounces: int = 0, aa: bool = False,
                   shadow_mode: int = RM_SHADOW_SOFT) -> rm_uniforms:
    """Synthetic frame of SURVEY 8(d); frame < 0 = default frame D."""
    u = rm_uniforms()
    _check(lib().rm_sweep_uniforms(frame, nframes, bounces, 1 if aa else 0, shadow_mode,
                                   C.byref(u)))
    return u


# ---- Camera (source/camera.hpp:12-35) --------------------------------------------------
class Camera:
    """Mirror of the reference ``Camera`` class (camera.hpp:12-35, camera.cpp:8-51)."""

    def __init__(self, width: int = 1024, height: int = 1024, mouseSensitivity: float = 1.0,
                 keyboardSpeed: float = 10.0, pos=(0.0, 0.0, 0.0), lookAt=(0.0, 0.0, -1.0),
                 up=(0.0, 1.0, 0.0)):
        self._s = rm_camera_state()
        f3 = C.c_float * 3
        _check(lib().rm_camera_init(C.byref(self._s), width, height, mouseSensitivity,
                                    keyboardSpeed, f3(*pos), f3(*lookAt), f3(*up)))

    def setMouse(self, x: float, y: float) -> None:  # camera.cpp:16-20
        _check(lib().rm_camera_set_mouse(C.byref(self._s), x, y))

    def lookAt(self, zN: bool = False, zP: bool = False, xN: bool = False, xP: bool = False,
               halfSpeed: bool = False, deltaTime: float = 0.0) -> None:  # camera.cpp:22-51
        _check(lib().rm_camera_look_at(C.byref(self._s), int(zN), int(zP), int(xN), int(xP),
                                       int(halfSpeed), deltaTime))

    def to_uniform(self) -> rm_camera:  # main.cpp:103-106
        c = rm_camera()
        _check(lib().rm_camera_to_uniform(C.byref(self._s), C.byref(c)))
        return c

    def __getattr__(self, name):
        s = object.__getattribute__(self, "_s")
        v = getattr(s, name)
        return tuple(v) if isinstance(v, C.Array) else v

    @property
    def state(self) -> rm_camera_state:
        return self._s


# ---- interactive input (main.cpp:20-39, 93-95, 155-234; MousePosition.cpp) -------------
class Input:
    """The reference's GLFW input globals and callbacks for one window.

    Owns the ``Camera`` the callbacks move (main.cpp:40's arguments by default) and the
    ``MouseInput`` angles.  A windowing front-end calls ``begin_frame(glfwGetTime())``,
    ``processInput(held)`` once per frame and forwards its key / cursor events to
    ``key_callback`` / ``mouse_callback``; ``to_uniforms`` then fills the per-frame uploads
    of main.cpp:101-120.  Every rule (diagonal half speed, bounce 0..5, PRESS-only toggles,
    first-mouse latch, float/double rounding) is librm's ``rm_input_*``.
    """

    def __init__(self, SCREEN_WIDTH: int = 1080, SCREEN_HEIGHT: int = 1080,
                 camera: Optional[Camera] = None):
        self._s = rm_input_state()
        _check(lib().rm_input_init(C.byref(self._s), SCREEN_WIDTH, SCREEN_HEIGHT))
        self.camera = camera if camera is not None else Camera(
            SCREEN_WIDTH, SCREEN_HEIGHT, 0.025, 10.0, (0, 0, 0), (0, 0, -1), (0, 1, 0))

    def begin_frame(self, now: float) -> None:  # main.cpp:93-95
        _check(lib().rm_input_begin_frame(C.byref(self._s), now))

    def processInput(self, held: int = 0) -> None:  # main.cpp:155-195
        """``held``: OR of HELD_* for the keys glfwGetKey reports as pressed."""
        _check(lib().rm_input_process(C.byref(self._s), held, C.byref(self.camera.state)))

    def key_callback(self, key: int, scancode: int = 0, action: int = PRESS,
                     mods: int = 0) -> None:  # main.cpp:197-217
        _check(lib().rm_input_key(C.byref(self._s), key, action))

    def mouse_callback(self, xpos: float, ypos: float) -> None:  # main.cpp:219-234
        _check(lib().rm_input_mouse(C.byref(self._s), xpos, ypos, C.byref(self.camera.state)))

    def EulerAngles(self) -> tuple:  # MousePosition.cpp:24-33
        out = (C.c_float * 3)()
        _check(lib().rm_input_euler_angles(C.byref(self._s), out))
        return tuple(out)

    def to_uniforms(self, u: Optional[rm_uniforms] = None) -> rm_uniforms:
        u = default_uniforms() if u is None else u
        _check(lib().rm_input_to_uniforms(C.byref(self._s), C.byref(self.camera.state),
                                          C.byref(u)))
        return u

    def __getattr__(self, name):
        return getattr(object.__getattribute__(self, "_s"), name)

    @property
    def state(self) -> rm_input_state:
        return self._s


# ---- Texture + compute program (texture.hpp:3-14, shader.hpp) ---------------------------
class Texture:
    """Mirror of the reference ``Texture`` (texture.hpp:3-14).

    ``GenerateTexture()`` creates the device image (a librm context);
    ``texOutput`` is the opaque handle that replaces the GL texture name.
    """

    def __init__(self, SCREEN_WIDTH: int = 720, SCREEN_HEIGHT: int = 720):
        self.texWidth = int(SCREEN_WIDTH)
        self.texHeight = int(SCREEN_HEIGHT)
        self.texOutput: Optional["Renderer"] = None

    def GenerateTexture(self, outputs: int = RM_OUT_RGBA8 | RM_OUT_RGBA32F,
                        kernel: int = RM_KERNEL_AUTO, device: int = -1) -> "Renderer":
        self.texOutput = Renderer(self.texWidth, self.texHeight, outputs=outputs, kernel=kernel,
                                  device=device)
        return self.texOutput


class Renderer:
    """One librm context: the compute program bound to its output image."""

    def __init__(self, width: int, height: int, *, outputs: int = RM_OUT_RGBA8,
                 kernel: int = RM_KERNEL_AUTO, counters: bool = False, device: int = -1,
                 row_block: int = 0, shard: int = 0, nshards: int = 1, ngpus: int = 0,
                 devices: Optional[Sequence[int]] = None, rank0_rows: int = 0,
                 shard_format: int = RM_SHARD_AUTO):
        """ngpus >= 1: one context over ngpus devices (`devices`, or device,
        device+1, ...), shards gathered with RCCL on the first (rm_config.ngpus).
        rank0_rows: shard 0's rows per round of the weighted interleave (0 = row_block).
        shard_format: RM_SHARD_* layout of the RGBA8 shard images (AUTO: packed RGB
        once the context gathers)."""
        devs = (C.c_int32 * len(devices))(*devices) if devices else None
        if devices:
            ngpus = len(devices)
        cfg = rm_config(struct_size=C.sizeof(rm_config), magic=RM_CONFIG_MAGIC, width=width, height=height,
                        device=device, outputs=outputs, kernel=kernel,
                        counters=1 if counters else 0, row_block=row_block, shard=shard,
                        nshards=nshards, rank0_rows=rank0_rows, shard_format=shard_format, ngpus=ngpus,
                        devices=C.cast(devs, C.POINTER(C.c_int32)) if devs else None)
        h = C.c_void_p()
        _check(lib().rm_create(C.byref(h), C.byref(cfg)))
        self._h = h
        self.width, self.height = width, height
        self.outputs = outputs if outputs else RM_OUT_RGBA8
        self.nshards, self.shard, self.row_block = max(nshards, 1), shard, row_block
        self.rank0_rows = rank0_rows
        self.shard_format = shard_format
        self.ngpus = ngpus
        self.rows = (shard_rows(height, row_block, nshards, shard, rank0_rows)[1]
                     if nshards > 1 and not ngpus else height)

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().rm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- uniforms by name (shader.hpp:19-69)
    def setBool(self, name: str, value: bool) -> int:
        return _check(lib().rm_set_bool(self._h, name.encode(), int(bool(value))), self._h)

    def setInt(self, name: str, value: int) -> int:
        return _check(lib().rm_set_int(self._h, name.encode(), int(value)), self._h)

    def setuInt(self, name: str, value: int) -> int:
        v = C.c_uint32(value)
        return _check(lib().rm_set_uint(self._h, name.encode(), C.byref(v)), self._h)

    def setFloat(self, name: str, value: float) -> int:
        return _check(lib().rm_set_float(self._h, name.encode(), float(value)), self._h)

    def setVec2(self, name: str, x, y=None) -> int:
        if y is None:
            x, y = x
        return _check(lib().rm_set_vec2(self._h, name.encode(), x, y), self._h)

    def setVec3(self, name: str, x, y=None, z=None) -> int:
        if y is None:
            x, y, z = x
        return _check(lib().rm_set_vec3(self._h, name.encode(), x, y, z), self._h)

    def setVec4(self, name: str, x, y=None, z=None, w=None) -> int:
        if y is None:
            x, y, z, w = x
        return _check(lib().rm_set_vec4(self._h, name.encode(), x, y, z, w), self._h)

    def set_scene(self, prims: Optional[Sequence[rm_primitive]]) -> None:
        """Render a runtime scene table from the next dispatch on (None: built-in scene)."""
        if prims is None:
            _check(lib().rm_set_scene(self.handle, None, 0), self.handle)
            return
        tbl = (rm_primitive * len(prims))(*prims)
        _check(lib().rm_set_scene(self.handle, tbl, len(prims)), self.handle)

    def specialize_scene(self, on: bool = True) -> None:
        """Render tables with kernels compiled for the table (hiprtc; rm_scene_specialize)."""
        _check(lib().rm_scene_specialize(self.handle, int(on)), self.handle)

    def scene_kernel_waves(self) -> int:
        """Waves per SIMD of the specialised table kernels in use (rm_scene_kernel_waves);
        0 = the generic table kernel or the built-in scene."""
        w = C.c_int32(0)
        _check(lib().rm_scene_kernel_waves(self.handle, C.byref(w)), self.handle)
        return int(w.value)

    def get_scene(self) -> list:
        n = C.c_int32(0)
        out = (rm_primitive * RM_MAX_PRIMITIVES)()
        _check(lib().rm_get_scene(self.handle, out, RM_MAX_PRIMITIVES, C.byref(n)), self.handle)
        return [out[i] for i in range(n.value)]

    def set_uniforms(self, u: rm_uniforms) -> None:
        _check(lib().rm_set_uniforms(self._h, C.byref(u)), self._h)

    def get_uniforms(self) -> rm_uniforms:
        u = rm_uniforms()
        _check(lib().rm_get_uniforms(self._h, C.byref(u)), self._h)
        return u

    # -- dispatch / barrier / readback
    def dispatch(self, u: Optional[rm_uniforms] = None) -> None:
        """glDispatchCompute (main.cpp:123): asynchronous."""
        if u is not None:
            self.set_uniforms(u)
        _check(lib().rm_dispatch(self._h), self._h)

    def dispatch_frames(self, frames: Sequence[rm_uniforms]) -> None:
        """Render len(frames) frames in one launch (rm_dispatch_frames): the images of
        set_uniforms + dispatch per frame; afterwards the image is the last frame's and
        read_frame_rgba8(k) reads frame k.  Asynchronous."""
        n = len(frames)
        arr = (rm_uniforms * n)(*frames)
        _check(lib().rm_dispatch_frames(self._h, arr, n), self._h)

    def read_frame_rgba8(self, k: int, flip_y: bool = False) -> np.ndarray:
        out = np.empty((self.rows, self.width, 4), np.uint8)
        _check(lib().rm_read_frame_rgba8(self._h, k, out.ctypes.data, 0, int(flip_y)), self._h)
        return out

    def read_frame_rgba32f(self, k: int, flip_y: bool = False) -> np.ndarray:
        out = np.empty((self.rows, self.width, 4), np.float32)
        _check(lib().rm_read_frame_rgba32f(self._h, k, out.ctypes.data, 0, int(flip_y)), self._h)
        return out

    def graph_enable(self, on: bool = True) -> None:
        """Switch to hipGraph replay of the frame (BASELINE cfg 5)."""
        _check(lib().rm_graph_enable(self._h, int(on)), self._h)

    def graph_dispatch(self, u: Optional[rm_uniforms] = None) -> None:
        """rm_dispatch through the captured graph (asynchronous)."""
        if u is not None:
            self.set_uniforms(u)
        _check(lib().rm_graph_dispatch(self._h), self._h)

    def synchronize(self) -> None:
        """glMemoryBarrier (main.cpp:125) + wait."""
        _check(lib().rm_synchronize(self._h), self._h)

    def read_rgba8(self, flip_y: bool = False) -> np.ndarray:
        out = np.empty((self.rows, self.width, 4), np.uint8)
        _check(lib().rm_read_rgba8(self._h, out.ctypes.data, 0, int(flip_y)), self._h)
        return out

    def read_rgba32f(self, flip_y: bool = False) -> np.ndarray:
        out = np.empty((self.rows, self.width, 4), np.float32)
        _check(lib().rm_read_rgba32f(self._h, out.ctypes.data, 0, int(flip_y)), self._h)
        return out

    def counters(self) -> dict:
        c = rm_counters()
        _check(lib().rm_get_counters(self._h, C.byref(c)), self._h)
        return c.as_dict()

    def sdf_counts(self) -> np.ndarray:
        out = np.empty((self.rows, self.width), np.uint32)
        _check(lib().rm_read_sdf_counts(self._h, out.ctypes.data), self._h)
        return out

    # -- device interop
    def set_stream(self, stream_ptr: Optional[int]) -> None:
        _check(lib().rm_set_stream(self._h, stream_ptr), self._h)

    def set_output_rgba8(self, device_ptr: Optional[int]) -> None:
        _check(lib().rm_set_output_rgba8(self._h, device_ptr), self._h)

    def output_rgba8_ptr(self) -> int:
        p = C.c_void_p()
        _check(lib().rm_get_output_rgba8(self._h, C.byref(p)), self._h)
        return p.value or 0

    def wait_output(self, stream_ptr: Optional[int]) -> None:
        """Order the caller's stream after every image write queued so far
        (rm_wait_output; a communicator batch assembles on an internal stream)."""
        _check(lib().rm_wait_output(self._h, stream_ptr), self._h)

    def unshard_rgba8(self, gathered_ptr: int, frame_ptr: int) -> None:
        _check(lib().rm_unshard_rgba8(self._h, gathered_ptr, frame_ptr), self._h)

    def unshard_batch_rgba8(self, gathered_ptr: int, k: int, n: int, frame_ptr: int) -> None:
        """Frame k of an n-frame batch gathered as [nshards][n][rows_cap][width]."""
        _check(lib().rm_unshard_batch_rgba8(self._h, gathered_ptr, k, n, frame_ptr), self._h)

    # -- one rank per process (rm_comm_init)
    def comm_init(self, comm_id: bytes, nranks: int, rank: int) -> None:
        """Join this shard context to an RCCL communicator: from then on dispatch
        renders, gathers on rank 0 and (rank 0) assembles the full frame."""
        buf = C.create_string_buffer(bytes(comm_id), COMM_ID_BYTES)
        _check(lib().rm_comm_init(self._h, buf, nranks, rank), self._h)
        if rank == 0:
            self.rows = self.height

    def comm_set_timeout(self, timeout_ms: int) -> None:
        """Deadline of rm_comm_init and of every later wait on this context (0: none)."""
        _check(lib().rm_comm_set_timeout(self._h, int(timeout_ms)), self._h)

    def comm_check(self) -> None:
        """Non-blocking health check of the communicator (raises RMError RM_ERR_COMM)."""
        _check(lib().rm_comm_check(self._h), self._h)

    def frame_phases(self) -> dict:
        """render / gather / assembly ms of the last timed eager dispatch (rm_frame_phases)."""
        r, g, a = C.c_double(0), C.c_double(0), C.c_double(0)
        _check(lib().rm_frame_phases(self._h, C.byref(r), C.byref(g), C.byref(a)), self._h)
        return {"render_ms": r.value, "gather_ms": g.value, "assemble_ms": a.value}

    def comm_info(self) -> tuple:
        r, n, g = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        _check(lib().rm_comm_info(self._h, C.byref(r), C.byref(n), C.byref(g)), self._h)
        return r.value, n.value, g.value

    def rccl_info(self) -> dict:
        """What RCCL itself reports for this context's communicator (rm_comm_rccl_info):
        ncclCommCount, ncclCommUserRank, ncclCommCuDevice, ncclGetVersion."""
        n, r, d, v = C.c_int32(0), C.c_int32(0), C.c_int32(0), C.c_int32(0)
        _check(lib().rm_comm_rccl_info(self._h, C.byref(n), C.byref(r), C.byref(d), C.byref(v)),
               self._h)
        return {"count": n.value, "user_rank": r.value, "hip_device": d.value, "version": v.value}

    def enable_timing(self, on: bool = True) -> None:
        _check(lib().rm_enable_timing(self._h, int(on)), self._h)

    def kernel_time_ms(self, reset: bool = False):
        ms = C.c_double(0.0)
        n = C.c_int64(0)
        _check(lib().rm_kernel_time_ms(self._h, C.byref(ms), C.byref(n), int(reset)), self._h)
        return ms.value, n.value


def comm_unique_id() -> bytes:
    """An RCCL unique id (ncclGetUniqueId) for rm_comm_init; rank 0 creates it and
    broadcasts it over the host's own channel."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().rm_comm_unique_id(buf, COMM_ID_BYTES))
    return buf.raw


# shader.hpp-style free functions over a Renderer ("program") ---------------------------
def CreateCompute(width: int, height: int, **kw) -> Renderer:  # shader.hpp:186-197
    return Renderer(width, height, **kw)


def useShader(program: Renderer) -> None:  # shader.hpp:17 (no global binding state)
    return None


def setBool(p: Renderer, name: str, v) -> int: return p.setBool(name, v)
def setInt(p: Renderer, name: str, v) -> int: return p.setInt(name, v)
def setuInt(p: Renderer, name: str, v) -> int: return p.setuInt(name, v)
def setFloat(p: Renderer, name: str, v) -> int: return p.setFloat(name, v)
def setVec2(p: Renderer, name: str, *v) -> int: return p.setVec2(name, *v)
def setVec3(p: Renderer, name: str, *v) -> int: return p.setVec3(name, *v)
def setVec4(p: Renderer, name: str, *v) -> int: return p.setVec4(name, *v)


def glDispatchCompute(p: Renderer) -> None:  # main.cpp:123
    p.dispatch()


def glMemoryBarrier(p: Renderer) -> None:  # main.cpp:125
    p.synchronize()


# ---- row sharding ---------------------------------------------------------
def shard_rows(height: int, row_block: int, nshards: int, shard: int = 0,
               rank0_rows: int = 0) -> tuple:
    """(real rows of `shard`, rows_cap) of the weighted interleave (rm_shard_rows)."""
    n, cap = C.c_int32(0), C.c_int32(0)
    _check(lib().rm_shard_rows(height, row_block, rank0_rows, nshards, shard, C.byref(n),
                               C.byref(cap)))
    return n.value, cap.value


def shard_rows_cap(height: int, row_block: int, nshards: int, rank0_rows: int = 0) -> int:
    return shard_rows(height, row_block, nshards, 0, rank0_rows)[1]


def shard_global_rows(height: int, row_block: int, shard: int, nshards: int,
                      rank0_rows: int = 0) -> np.ndarray:
    """Global row of every local row of `shard` (-1: padding), rm_shard_to_global."""
    cap = shard_rows_cap(height, row_block, nshards, rank0_rows)
    return np.array([lib().rm_shard_to_global(height, row_block, rank0_rows, nshards, shard, r)
                     for r in range(cap)], np.int32)


def shard_owner(height: int, row_block: int, nshards: int, row: int, rank0_rows: int = 0) -> tuple:
    """(shard, local row) holding global row `row` (rm_shard_owner)."""
    s, l = C.c_int32(0), C.c_int32(0)
    _check(lib().rm_shard_owner(height, row_block, rank0_rows, nshards, row, C.byref(s), C.byref(l)))
    return s.value, l.value


def best_rank0_rows(row_block: int, nshards: int, assemble_ratio: float) -> int:
    """Shard 0's rows per round that balance its render + the frame's assembly against
    the other shards' render: the r0 in 1..2 row_block minimising
    max(r0 / P + a, row_block / P), P = r0 + (nshards - 1) row_block, with a = the
    assembly's time over one GPU's render time of the whole frame."""
    if nshards <= 1:
        return 0
    best, arg = None, row_block
    for r0 in range(1, 2 * row_block + 1):
        P = r0 + (nshards - 1) * row_block
        t = max(r0 / P + assemble_ratio, row_block / P)
        if best is None or t < best - 1e-12:
            best, arg = t, r0
    return arg


def quantize_rgba8(img: np.ndarray) -> np.ndarray:
    """round(clamp(c,0,1)*255) in float32, NaN -> 0."""
    c = img.astype(np.float32)
    v = np.where(c > 0, np.where(c < 1, c, np.float32(1)), np.float32(0)).astype(np.float32)
    return (v * np.float32(255) + np.float32(0.5)).astype(np.uint8)


def write_ppm(path: str, rgba8_top_first: np.ndarray) -> None:
    """Write an RGBA8 image (top row first) as binary PPM."""
    h, w = rgba8_top_first.shape[:2]
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(rgba8_top_first[..., :3]).tobytes())
