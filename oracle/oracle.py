"""ctypes binding of the CPU oracle (oracle/rm_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / CPU baseline.  librm (the product) never
loads the oracle.  See rm_oracle.h for what the oracle is pinned against.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
# RM_ORACLE selects another build of the same source (the sanitizer build, `make asan`)
ORACLE_SO = os.environ.get("RM_ORACLE", os.path.join(_HERE, "_build", "librm_oracle.so"))

sys.path.insert(0, os.path.join(_ROOT, "opengl-raymarching-in-compute-shader_amd"))
from rmarch import rm_counters, rm_primitive, rm_uniforms  # noqa: E402  (shared POD structs)


class rmo_hit(C.Structure):
    _fields_ = [("hitpoint", C.c_float), ("color", C.c_float * 3), ("id", C.c_int32),
                ("material", C.c_float)]


_lib: Optional[C.CDLL] = None
_F3 = C.c_float * 3
_PU = C.POINTER(rm_uniforms)


def build() -> str:
    """Compile the oracle with the committed recipe (Makefile target `oracle`)."""
    subprocess.run(["make", "-s", "oracle"], cwd=_ROOT, check=True)
    return ORACLE_SO


# Compiler flags of the committed recipe (Makefile OFLAGS): no FMA contraction and
# no fast-math, so every float op is one IEEE op in GLSL source order.
OFLAGS = ["-std=c11", "-O3", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC"]


def build_native(outdir: str) -> str:
    """The BASELINE.md `-march=native` variant (contraction still off), compiled
    for THIS host's CPU into `outdir` (bench.py builds it on the machine it runs
    on; a binary built for another CPU could use instructions this one lacks)."""
    os.makedirs(outdir, exist_ok=True)
    out = os.path.join(outdir, "librm_oracle_native.so")
    subprocess.run(["gcc", *OFLAGS, "-march=native", "-shared", "-o", out,
                    os.path.join(_HERE, "rm_oracle.c"), "-lm"], check=True)
    return out


def _bind(L: C.CDLL) -> C.CDLL:
    L.rmo_render.restype = C.c_int
    L.rmo_render.argtypes = [_PU, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                             C.c_void_p, C.c_void_p, C.POINTER(rm_counters),
                             C.POINTER(rm_counters), C.c_int32]
    L.rmo_render_scene.restype = C.c_int
    L.rmo_render_scene.argtypes = [_PU, C.POINTER(rm_primitive), C.c_int32, C.c_int32,
                                   C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.POINTER(rm_counters),
                                   C.POINTER(rm_counters), C.c_int32]
    L.rmo_sdf.argtypes = [_PU, _F3, C.POINTER(rmo_hit)]
    L.rmo_raymarch.argtypes = [_PU, _F3, _F3, C.c_int32, C.POINTER(rmo_hit),
                               C.POINTER(C.c_uint32)]
    L.rmo_get_normal.argtypes = [_PU, _F3, _F3]
    L.rmo_softshadow.restype = C.c_float
    L.rmo_softshadow.argtypes = [_PU, _F3, _F3, C.c_float, C.POINTER(C.c_uint32)]
    L.rmo_point_light.argtypes = [_PU, _F3, _F3, _F3, _F3]
    L.rmo_cast_ray.argtypes = [_PU, C.c_float, C.c_float, _F3, _F3]
    L.rmo_render_ray.argtypes = [_PU, _F3, _F3, _F3]
    L.rmo_pixel.argtypes = [_PU, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                            C.c_float * 4]
    L.rmo_quantize.restype = C.c_uint8
    L.rmo_quantize.argtypes = [C.c_float]
    L.rmo_max_threads.restype = C.c_int
    return L


def load(path: str) -> C.CDLL:
    """Load an oracle build other than the default one (e.g. build_native's)."""
    return _bind(C.CDLL(path))


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        _lib = _bind(C.CDLL(ORACLE_SO))
    return _lib


def render(u: rm_uniforms, W: int, H: int, rows: Optional[Sequence[int]] = None,
           nthreads: int = 0, want_f32: bool = True, want_counts: bool = True,
           scene: Optional[Sequence[rm_primitive]] = None, L: Optional[C.CDLL] = None) -> dict:
    """Render rows (default: all) with the oracle.  Row 0 = bottom (py = 0).

    ``scene``: a runtime scene table (rm_primitive entries) in place of the GLSL's
    own sdf() (rmo_render_scene)."""
    n = H if rows is None else len(rows)
    rows_arr = None if rows is None else np.ascontiguousarray(rows, np.int32)
    rgba8 = np.zeros((n, W, 4), np.uint8)
    f32 = np.zeros((n, W, 4), np.float32) if want_f32 else None
    counts = np.zeros((n, W), np.uint32) if want_counts else None
    cnt, full = rm_counters(), rm_counters()
    tail = (W, H, None if rows_arr is None else rows_arr.ctypes.data, n,
            None if f32 is None else f32.ctypes.data, rgba8.ctypes.data,
            None if counts is None else counts.ctypes.data, C.byref(cnt), C.byref(full), nthreads)
    L = L or lib()
    if scene is None:
        rc = L.rmo_render(C.byref(u), *tail)
    else:
        tbl = (rm_primitive * len(scene))(*scene)
        rc = L.rmo_render_scene(C.byref(u), tbl, len(scene), *tail)
    if rc != 0:
        raise ValueError("rmo_render: bad arguments")
    return {"rgba8": rgba8, "rgba32f": f32, "sdf_counts": counts, "counters": cnt.as_dict(),
            "full_counters": full.as_dict()}


def sdf(u: rm_uniforms, pos) -> rmo_hit:
    h = rmo_hit()
    lib().rmo_sdf(C.byref(u), _F3(*pos), C.byref(h))
    return h


def raymarch(u: rm_uniforms, ro, rd, reflected: bool = False):
    h = rmo_hit()
    steps = C.c_uint32(0)
    lib().rmo_raymarch(C.byref(u), _F3(*ro), _F3(*rd), int(reflected), C.byref(h),
                       C.byref(steps))
    return h, steps.value


def get_normal(u: rm_uniforms, pos) -> np.ndarray:
    out = _F3()
    lib().rmo_get_normal(C.byref(u), _F3(*pos), out)
    return np.array(out, np.float32)


def softshadow(u: rm_uniforms, ro, rd, k: float):
    steps = C.c_uint32(0)
    r = lib().rmo_softshadow(C.byref(u), _F3(*ro), _F3(*rd), k, C.byref(steps))
    return r, steps.value


def point_light(u: rm_uniforms, color, normal, pos) -> np.ndarray:
    out = _F3()
    lib().rmo_point_light(C.byref(u), _F3(*color), _F3(*normal), _F3(*pos), out)
    return np.array(out, np.float32)


def cast_ray(u: rm_uniforms, uvx: float, uvy: float):
    ro, rd = _F3(), _F3()
    lib().rmo_cast_ray(C.byref(u), uvx, uvy, ro, rd)
    return np.array(ro, np.float32), np.array(rd, np.float32)


def render_ray(u: rm_uniforms, ro, rd) -> np.ndarray:
    out = _F3()
    lib().rmo_render_ray(C.byref(u), _F3(*ro), _F3(*rd), out)
    return np.array(out, np.float32)


def pixel(u: rm_uniforms, W: int, H: int, px: int, py: int) -> np.ndarray:
    out = (C.c_float * 4)()
    lib().rmo_pixel(C.byref(u), W, H, px, py, out)
    return np.array(out, np.float32)


def quantize(c: float) -> int:
    return int(lib().rmo_quantize(c))


def max_threads() -> int:
    return int(lib().rmo_max_threads())
