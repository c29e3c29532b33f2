"""Scene and camera inputs of the render loop (Globals.hpp:8-37, SceneGenerators.hpp).

A Scene is the reference's structure-of-arrays (g_spheres, g_radii, g_colors,
g_materials, g_diffuses).  Generators run in the native library
(spt_scene_* in include/spt_hip.h) with an explicit seed instead of the clock.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native

# Material, Definitions.hpp:7-13
SKYBOX, REFLECTIVE, REFRACTIVE, DIFFUSE = 0, 1, 2, 3

# Globals.hpp:21-29 defaults
DEFAULT_EYE = (0.0, 1.0, -3.0, 0.0)
DEFAULT_LOOK_AT = (0.0, 1.0, 0.0, 0.0)
DEFAULT_UP = (0.0, 1.0, 0.0, 0.0)
INIT_COLOR = (137.0, 207.0, 240.0, 0.0)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class Scene:
    centers: np.ndarray    # (n, 4) float32, w = 0
    radii: np.ndarray      # (n,) float32
    colors: np.ndarray     # (n, 4) float32, 0..255 scale
    materials: np.ndarray  # (n,) uint8
    fuzz: np.ndarray       # (n,) float32 (g_diffuses)

    def __post_init__(self):
        n = len(self.radii)
        self.centers = np.ascontiguousarray(np.asarray(self.centers, np.float32).reshape(n, 4))
        self.radii = np.ascontiguousarray(np.asarray(self.radii, np.float32).reshape(n))
        self.colors = np.ascontiguousarray(np.asarray(self.colors, np.float32).reshape(n, 4))
        self.materials = np.ascontiguousarray(np.asarray(self.materials, np.uint8).reshape(n))
        self.fuzz = np.ascontiguousarray(np.asarray(self.fuzz, np.float32).reshape(n))

    @property
    def n(self) -> int:
        return int(len(self.radii))

    def save(self, path: str) -> None:
        np.savez(path, centers=self.centers, radii=self.radii, colors=self.colors, materials=self.materials,
                 fuzz=self.fuzz)

    @classmethod
    def load(cls, path: str) -> "Scene":
        z = np.load(path, allow_pickle=False)
        return cls(z["centers"], z["radii"], z["colors"], z["materials"], z["fuzz"])


def _alloc(cap: int):
    return (np.zeros((cap, 4), np.float32), np.zeros(cap, np.float32), np.zeros((cap, 4), np.float32),
            np.zeros(cap, np.uint8), np.zeros(cap, np.float32))


def generate_spheres(seed: int = 1, capacity: int = 4096, z_end: float = 20.0) -> Scene:
    """GenerateSpheres (SceneGenerators.hpp:6-66), the RANDOM scene (~140-160 spheres).
    z_end: the row loop's bound (SceneGenerators.hpp:32, the reference's 20); 37.5 gives
    BASELINE.json's "~500-sphere" scene (488 spheres for seed 1)."""
    c, r, col, m, f = _alloc(capacity)
    n = ctypes.c_uint32(0)
    if z_end == 20.0:
        _native.check(_native.lib().spt_scene_generate_random(seed, capacity, _p(c), _p(r), _p(col), _p(m), _p(f),
                                                              ctypes.byref(n)))
    else:
        _native.check(_native.lib().spt_scene_generate_random_rows(seed, ctypes.c_float(z_end), capacity, _p(c), _p(r),
                                                                   _p(col), _p(m), _p(f), ctypes.byref(n)))
    k = n.value
    return Scene(c[:k], r[:k], col[:k], m[:k], f[:k])


def init_spheres(seed: int = 1) -> Scene:
    """InitSpheres (SceneGenerators.hpp:68-133), the REFERENCE scene (10 spheres)."""
    c, r, col, m, f = _alloc(10)
    n = ctypes.c_uint32(0)
    _native.check(_native.lib().spt_scene_init_reference(seed, _p(c), _p(r), _p(col), _p(m), _p(f),
                                                         ctypes.byref(n)))
    return Scene(c, r, col, m, f)


def generate_stress(seed: int, n: int) -> Scene:
    """Build-side n-sphere stress scene (BASELINE config 5; n > 255 needs the 32-bit index)."""
    c, r, col, m, f = _alloc(n)
    _native.check(_native.lib().spt_scene_generate_stress(seed, n, _p(c), _p(r), _p(col), _p(m), _p(f)))
    return Scene(c, r, col, m, f)


def cornell3() -> Scene:
    """BASELINE config 1's "3-sphere" scene as SURVEY.md §8d defines it: the
    InitSpheres ground plus a diffuse, a mirror (fuzz 0) and a glass sphere."""
    ref = init_spheres(1)
    idx = [0, 1, 2, 3]
    mats = np.array([DIFFUSE, DIFFUSE, REFLECTIVE, REFRACTIVE], np.uint8)
    fuzz = np.array([0.0, 0.0, 0.0, 0.0], np.float32)
    return Scene(ref.centers[idx], ref.radii[idx], ref.colors[idx], mats, fuzz)


def camera_basis(eye=DEFAULT_EYE, look_at=DEFAULT_LOOK_AT, up=DEFAULT_UP) -> np.ndarray:
    """viewMatrix = Transpose(CreateCameraBasisMatrix(eye, lookAt, up)) (Renderer.hpp:321)."""
    out = np.zeros(16, np.float32)
    e, l, u = (np.asarray(v, np.float32) for v in (eye, look_at, up))
    _native.check(_native.lib().spt_camera_basis(_p(e), _p(l), _p(u), _p(out)))
    return out
