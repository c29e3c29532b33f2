"""ctypes binding of the CPU restatement (oracle/spt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See spt_oracle.h for
the parity status ("parity unpinned" end to end; building blocks pinned by KATs).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libspt_oracle.so")

SKYBOX, REFLECTIVE, REFRACTIVE, DIFFUSE = 0, 1, 2, 3


class Scene(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32),
        ("centers", ctypes.c_void_p),
        ("radii", ctypes.c_void_p),
        ("colors", ctypes.c_void_p),
        ("materials", ctypes.c_void_p),
        ("fuzz", ctypes.c_void_p),
    ]


class Frame(ctypes.Structure):
    _fields_ = [
        ("view", ctypes.c_float * 16),
        ("eye", ctypes.c_float * 4),
        ("sky", ctypes.c_float * 4),
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("spp", ctypes.c_uint32),
        ("bounces", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
    ]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        u32, u64, f32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float
        L.spo_next_u32.argtypes = [P]; L.spo_next_u32.restype = u32
        L.spo_uniform.argtypes = [P, f32, f32]; L.spo_uniform.restype = f32
        L.spo_uniform_u32.argtypes = [u32, f32, f32]; L.spo_uniform_u32.restype = f32
        L.spo_sample_key.argtypes = [u64, u32, u32]; L.spo_sample_key.restype = u64
        L.spo_scene_state.argtypes = [u32]; L.spo_scene_state.restype = u64
        L.spo_ball_vector.argtypes = [P, P]; L.spo_ball_vector.restype = None
        L.spo_camera_basis.argtypes = [P, P, P, P]; L.spo_camera_basis.restype = None
        L.spo_find_closest.argtypes = [P, P, P]; L.spo_find_closest.restype = u32
        L.spo_write_pixel.argtypes = [P, P]; L.spo_write_pixel.restype = None
        L.spo_trace_sample.argtypes = [P, P, u32, u32, u32, ctypes.c_int, P]; L.spo_trace_sample.restype = u32
        L.spo_primary_winners.argtypes = [P, P, P, u32, P]; L.spo_primary_winners.restype = None
        for fn in (L.spo_render_segment, L.spo_render_segment_task):
            fn.argtypes = [P, P, u32, u32, u32, u32, P, P]; fn.restype = u64
        L.spo_render_image_parallel.argtypes = [P, P, u32, ctypes.c_int, P, P]
        L.spo_render_image_parallel.restype = ctypes.c_int
        L.spo_generate_spheres.argtypes = [u32, u32, P, P, P, P, P]; L.spo_generate_spheres.restype = u32
        L.spo_init_spheres.argtypes = [u32, P, P, P, P, P]; L.spo_init_spheres.restype = u32
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleScene:
    """Keeps numpy arrays alive behind a spo_scene struct."""

    def __init__(self, centers, radii, colors, materials, fuzz):
        n = len(radii)
        self.centers = np.ascontiguousarray(np.asarray(centers, np.float32).reshape(n, 4))
        self.radii = np.ascontiguousarray(np.asarray(radii, np.float32).reshape(n))
        self.colors = np.ascontiguousarray(np.asarray(colors, np.float32).reshape(n, 4))
        self.materials = np.ascontiguousarray(np.asarray(materials, np.uint8).reshape(n))
        self.fuzz = np.ascontiguousarray(np.asarray(fuzz, np.float32).reshape(n))
        self.s = Scene(n, _p(self.centers), _p(self.radii), _p(self.colors), _p(self.materials), _p(self.fuzz))

    @property
    def ref(self):
        return ctypes.byref(self.s)


def make_frame(view, eye, sky, width, height, spp, bounces, seed) -> Frame:
    f = Frame()
    f.view[:] = [float(v) for v in np.asarray(view, np.float32).reshape(16)]
    f.eye[:] = [float(v) for v in np.asarray(eye, np.float32).reshape(4)]
    f.sky[:] = [float(v) for v in np.asarray(sky, np.float32).reshape(4)]
    f.width, f.height, f.spp, f.bounces, f.seed = width, height, spp, bounces, seed
    return f


def generate_spheres(seed: int, cap: int = 4096):
    c = np.zeros((cap, 4), np.float32); r = np.zeros(cap, np.float32); col = np.zeros((cap, 4), np.float32)
    m = np.zeros(cap, np.uint8); fz = np.zeros(cap, np.float32)
    n = lib().spo_generate_spheres(seed, cap, _p(c), _p(r), _p(col), _p(m), _p(fz))
    return OracleScene(c[:n], r[:n], col[:n], m[:n], fz[:n])


def init_spheres(seed: int):
    c = np.zeros((10, 4), np.float32); r = np.zeros(10, np.float32); col = np.zeros((10, 4), np.float32)
    m = np.zeros(10, np.uint8); fz = np.zeros(10, np.float32)
    n = lib().spo_init_spheres(seed, _p(c), _p(r), _p(col), _p(m), _p(fz))
    return OracleScene(c[:n], r[:n], col[:n], m[:n], fz[:n])


def camera_basis(eye, look_at, up):
    out = np.zeros(16, np.float32)
    e = np.asarray(eye, np.float32); l = np.asarray(look_at, np.float32); u = np.asarray(up, np.float32)
    lib().spo_camera_basis(_p(e), _p(l), _p(u), _p(out))
    return out


def render_segment(scene: OracleScene, frame: Frame, yB, yE, xB, xE, task=False, rgb8=None):
    rgba = np.zeros(((yE - yB) * (xE - xB), 4), np.float32)
    fn = lib().spo_render_segment_task if task else lib().spo_render_segment
    casts = fn(scene.ref, ctypes.byref(frame), yB, yE, xB, xE, _p(rgba), _p(rgb8) if rgb8 is not None else None)
    return rgba, casts


def render_image_parallel(scene: OracleScene, frame: Frame, thread_count: int, mode: int = 0, want_rgba=True):
    rgba = np.zeros((frame.height * frame.width, 4), np.float32) if want_rgba else None
    rgb8 = np.zeros(frame.width * frame.height * 3, np.uint8)
    rc = lib().spo_render_image_parallel(scene.ref, ctypes.byref(frame), thread_count, mode,
                                         _p(rgba) if rgba is not None else None, _p(rgb8))
    if rc != 0:
        raise RuntimeError("spo_render_image_parallel failed")
    return rgba, rgb8


def trace_sample(scene: OracleScene, frame: Frame, x, y, s, task=False):
    out = np.zeros(4, np.float32)
    casts = lib().spo_trace_sample(scene.ref, ctypes.byref(frame), x, y, s, int(task), _p(out))
    return out, casts


def primary_winners(scene: OracleScene, frame: Frame, xys) -> np.ndarray:
    """Closest sphere (index; scene.n = none) of the primary ray of each (x, y, s) row."""
    xys = np.ascontiguousarray(xys, np.uint32)
    out = np.zeros(len(xys), np.uint32)
    lib().spo_primary_winners(scene.ref, ctypes.byref(frame), _p(xys), len(xys), _p(out))
    return out
