"""Host-side mirror of the reference's render entry points over the HIP C ABI.

Reference interface (all state in globals, Globals.hpp:8-37):

    void RenderSegment(RenderSegmentData)       SingleThreadPathTracer.hpp:114-137
    void RenderSegmentTask(RenderSegmentData)   TaskBasedPathTracer.hpp:54-206
    RenderImageParallelMain()                   Renderer.hpp:257-302 (tile dispatch)
    RenderImage()                               Renderer.hpp:304-308

Here the globals live in a `Globals` object that owns a device context; the two
entry points keep their names and argument meaning (a pixel rectangle) and write
the reference's g_data byte layout.  Errors raise SptError (the reference has no
error channel).
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _native
from .scene import INIT_COLOR, DEFAULT_EYE, DEFAULT_LOOK_AT, DEFAULT_UP, Scene, camera_basis


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


_PROGRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32)


@dataclass
class RenderSegmentData:
    """Definitions.hpp:15-21."""
    yBegin: int = 0
    yEnd: int = 0
    xBegin: int = 0
    xEnd: int = 0


class Context:
    """One device context (spt_ctx) holding scene, camera and config."""

    def __init__(self, device: int = 0, devices=None):
        """One device, or with `devices` (a list of ordinals, repeats allowed) a
        multi-device context (spt_ctx_create_multi) whose member 0 is devices[0]."""
        L = _native.lib()
        h = ctypes.c_void_p()
        if devices is None:
            _native.check(L.spt_ctx_create(device, ctypes.byref(h)))
            self.devices = [device]
        else:
            devs = np.ascontiguousarray(np.asarray(devices, np.int32))
            _native.check(L.spt_ctx_create_multi(_p(devs), len(devs), ctypes.byref(h)))
            self.devices = [int(d) for d in devs]
        self._h = h
        self.device = self.devices[0]
        self._frame = None  # (width, height) after set_params

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            _native.lib().spt_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, code: int) -> None:
        _native.check(code, self._h)

    def set_scene(self, scene: Scene) -> None:
        self._scene = scene  # keep arrays alive for the duration of the call
        self._check(_native.lib().spt_set_scene(self._h, _p(scene.centers), _p(scene.radii), _p(scene.colors),
                                                _p(scene.materials), _p(scene.fuzz), scene.n))

    def set_camera(self, view, eye=DEFAULT_EYE, sky=INIT_COLOR) -> None:
        v = np.ascontiguousarray(np.asarray(view, np.float32).reshape(16))
        e = np.ascontiguousarray(np.asarray(eye, np.float32).reshape(4))
        s = np.ascontiguousarray(np.asarray(sky, np.float32).reshape(4))
        self._check(_native.lib().spt_set_camera(self._h, _p(v), _p(e), _p(s)))

    def set_params(self, width: int, height: int, spp: int, bounces: int, seed: int = 1) -> None:
        self._check(_native.lib().spt_set_params(self._h, width, height, spp, bounces, seed))
        self._frame = (width, height)

    def set_cluster_size(self, k: int) -> None:
        """Culling cluster size (0 = brute force over every sphere); results identical."""
        self._check(_native.lib().spt_set_cluster_size(self._h, int(k)))

    def set_cluster_tree(self, branching: int) -> None:
        """Children per inner node of the cluster tree (0 = flat list,
        _native.TREE_AUTO = default heuristic); results identical."""
        self._check(_native.lib().spt_set_cluster_tree(self._h, int(branching)))

    def prepare_dropin(self) -> None:
        """spt_prepare_dropin (what the C++ shim does once after creating its context): create
        the drop-in's batch and read-ahead streams now, and arm the tiling read-ahead at a
        tiling's first call (SPT_READAHEAD_FIRST=0: only after a whole tiling)."""
        self._check(_native.lib().spt_prepare_dropin(self._h))

    def set_reserved_cus(self, n: int) -> None:
        """Keep n CUs free of launched renders (spt_set_reserved_cus: 32 = one per shader
        engine lets a whole-CU kernel on another stream start beside a render); results
        identical."""
        self._check(_native.lib().spt_set_reserved_cus(self._h, int(n)))

    def set_engine(self, engine: int) -> None:
        """_native.ENGINE_MEGAKERNEL (default) or _native.ENGINE_WAVEFRONT; results identical."""
        self._check(_native.lib().spt_set_engine(self._h, int(engine)))

    def set_workspace(self, nbytes: int) -> None:
        self._check(_native.lib().spt_set_workspace(self._h, int(nbytes)))

    def render_segment(self, yB, yE, xB, xE, g_data=None, task=False, rgba=True):
        """Returns region-local float4 pixels (None with rgba=False: g_data only, the C++
        drop-in's form, which the tiling read-ahead serves); writes g_data bytes of the
        region if given."""
        out = np.zeros((max(yE - yB, 0) * max(xE - xB, 0), 4), np.float32) if rgba else None
        fn = _native.lib().spt_render_segment_task if task else _native.lib().spt_render_segment
        gp = None
        if g_data is not None:
            assert g_data.dtype == np.uint8 and g_data.flags.c_contiguous
            gp = _p(g_data)
        self._check(fn(self._h, yB, yE, xB, xE, _p(out) if rgba else None, gp))
        return out

    def render_frame(self, g_data=None, task=False, rgba=True):
        """The whole frame over every member device (spt_render_frame): returns the
        row-major float4 frame (or None with rgba=False); writes g_data if given."""
        L = _native.lib()
        if self._frame is None:
            # SPT_ERR_STATE, as the library reports it to its own callers
            raise _native.SptError(2, "params not set (set_params)")
        w, h = self._frame
        out = np.zeros((w * h, 4), np.float32) if rgba else None
        gp = None
        if g_data is not None:
            assert g_data.dtype == np.uint8 and g_data.flags.c_contiguous and g_data.size == w * h * 3
            gp = _p(g_data)
        self._check(L.spt_render_frame(self._h, 1 if task else 0, _p(out) if rgba else None, gp))
        return out

    def pin_host(self, arr: np.ndarray) -> None:
        """Page-lock a host array (e.g. g_data) for direct device-to-host copies."""
        assert arr.flags.c_contiguous
        self._check(_native.lib().spt_pin_host(self._h, _p(arr), arr.nbytes))

    def unpin_host(self, arr: np.ndarray) -> None:
        self._check(_native.lib().spt_unpin_host(self._h, _p(arr)))

    def render_progressive(self, yB, yE, xB, xE, pass_spp: int, g_data=None, callback=None, task=False):
        """Progressive render in passes of pass_spp samples.  After each pass the returned
        float4 array (and g_data, if given) hold the render at the samples done so far
        (bit-identical to a render with that many samples) and callback(samples_done)
        runs; a truthy return stops the render."""
        rgba = np.zeros((max(yE - yB, 0) * max(xE - xB, 0), 4), np.float32)
        gp = None
        if g_data is not None:
            assert g_data.dtype == np.uint8 and g_data.flags.c_contiguous
            gp = _p(g_data)
        errors = []

        def tramp(_user, done):
            try:
                return 1 if (callback is not None and callback(int(done))) else 0
            except BaseException as e:  # stop the render, re-raise below
                errors.append(e)
                return 1

        cb = _PROGRESS_FN(tramp)
        self._check(_native.lib().spt_render_progressive(self._h, int(task), yB, yE, xB, xE, pass_spp, _p(rgba), gp,
                                                         ctypes.cast(cb, ctypes.c_void_p), None))
        if errors:
            raise errors[0]
        return rgba

    def render_samples(self, yB, yE, xB, xE, spp: int, task=False) -> np.ndarray:
        out = np.zeros(((yE - yB) * (xE - xB), spp, 4), np.float32)
        self._check(_native.lib().spt_render_samples(self._h, int(task), yB, yE, xB, xE, _p(out)))
        return out

    def render_rows_async(self, mode, yB, yE, strip, parts, part, xB, xE, d_rgba=0, d_rgb8=0, stream=0) -> None:
        """Device-resident launch; d_rgba/d_rgb8/stream are raw device pointers / hipStream_t."""
        self._check(_native.lib().spt_render_rows_async(self._h, mode, yB, yE, strip, parts, part, xB, xE,
                                                        ctypes.c_void_p(d_rgba or None),
                                                        ctypes.c_void_p(d_rgb8 or None),
                                                        ctypes.c_void_p(stream or None)))

    def assemble_rows_async(self, d_tiles, max_rows, yB, yE, strip, parts, xB, xE, d_frame=0, d_rgb8=0,
                            stream=0) -> None:
        self._check(_native.lib().spt_assemble_rows_async(self._h, ctypes.c_void_p(d_tiles), max_rows, yB, yE, strip,
                                                          parts, xB, xE, ctypes.c_void_p(d_frame or None),
                                                          ctypes.c_void_p(d_rgb8 or None),
                                                          ctypes.c_void_p(stream or None)))

    def render_task_range_async(self, i0, i1, d_rgba, stream=0) -> None:
        """Outputs [i0, i1) of RenderSegmentTask({0, H, 0, W}) on a non-square frame into
        d_rgba (spt_render_task_range_async: the rank-share form of its aliasing)."""
        self._check(_native.lib().spt_render_task_range_async(self._h, i0, i1, ctypes.c_void_p(d_rgba or None),
                                                              ctypes.c_void_p(stream or None)))

    def synchronize(self) -> None:
        self._check(_native.lib().spt_synchronize(self._h))

    def service_start(self) -> None:
        """Render through the resident render service (spt_service_start): consecutive
        renders run as jobs of one persistent launch, without a ramp and tail each."""
        self._check(_native.lib().spt_service_start(self._h))

    def service_set_full_grid(self, full: bool) -> None:
        """Sessions on every block slot (True) or one per CU left free (False, the default)."""
        self._check(_native.lib().spt_service_set_full_grid(self._h, 1 if full else 0))

    def service_stop(self) -> None:
        """Drain and end the service session; renders launch per call again."""
        self._check(_native.lib().spt_service_stop(self._h))

    def stats(self) -> dict:
        s = _native.Stats()
        self._check(_native.lib().spt_get_stats(self._h, ctypes.byref(s)))
        d = {k: getattr(s, k) for k, _ in _native.Stats._fields_}
        d["diag"] = list(s.diag)
        return d

    def reset_stats(self) -> None:
        self._check(_native.lib().spt_reset_stats(self._h))

    def selftest_numerics(self, a, b, bits) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        bits = np.ascontiguousarray(bits, np.uint32)
        out = np.zeros((len(a), _native.SELFTEST_COLS), np.float32)
        self._check(_native.lib().spt_selftest_numerics(self._h, _p(a), _p(b), _p(bits), len(a), _p(out)))
        return out


def task_range(width, height, parts, part) -> tuple[int, int]:
    """Part `part` of `parts`'s outputs [i0, i1) of a non-square task-mode frame (spt_task_range)."""
    a, b = ctypes.c_uint32(), ctypes.c_uint32()
    _native.check(_native.lib().spt_task_range(width, height, parts, part, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def rows_count(yB, yE, strip, parts, part) -> int:
    r = ctypes.c_uint32(0)
    _native.check(_native.lib().spt_rows_count(yB, yE, strip, parts, part, ctypes.byref(r)))
    return r.value


class Globals:
    """The reference's global state (Globals.hpp:8-37) bound to a device context.

    g_width/g_height/g_samples/g_bounces, the scene SoA, viewMatrix/eyePos/
    initColor and the g_data framebuffer (RGB8, g_width*g_height*3 bytes).
    """

    def __init__(self, scene: Scene, width=1440, height=1440, samples=100, bounces=10, seed=1, eye=DEFAULT_EYE,
                 look_at=DEFAULT_LOOK_AT, up=DEFAULT_UP, init_color=INIT_COLOR, device=0, context=None,
                 devices=None):
        self.g_width, self.g_height, self.g_samples, self.g_bounces = width, height, samples, bounces
        self.g_stride = 3
        self.g_size = width * height * 3
        self.g_data = np.zeros(self.g_size, np.uint8)
        self.eyePos, self.lookAt, self.upDir, self.initColor = eye, look_at, up, init_color
        self.viewMatrix = camera_basis(eye, look_at, up)
        self.scene = scene
        self.seed = seed
        self.ctx = context or Context(device, devices=devices)
        self._lock = threading.Lock()
        self.sync()

    def sync(self) -> None:
        """Push the current globals to the device context."""
        self.ctx.set_scene(self.scene)
        self.ctx.set_camera(self.viewMatrix, self.eyePos, self.initColor)
        self.ctx.set_params(self.g_width, self.g_height, self.g_samples, self.g_bounces, self.seed)


def SaveImage(g: Globals, directory: str = ".") -> str:
    """io::SaveImage (IOHelpers.hpp:24-27): g_data as a 24-bit BMP named
    output{g_samples}s{g_bounces}b.bmp, in stbi_write_bmp's layout; returns the path."""
    import os
    path = os.path.join(directory, f"output{g.g_samples}s{g.g_bounces}b.bmp")
    data = np.ascontiguousarray(g.g_data, np.uint8)
    _native.check(_native.lib().spt_save_bmp(path.encode(), g.g_width, g.g_height, g.g_stride, _p(data)))
    return path


def RenderSegment(segment: RenderSegmentData, g: Globals) -> np.ndarray:
    """SingleThreadPathTracer.hpp:114-137: render the rectangle into g.g_data.
    Returns the float pixel colours (region-local, the value io::WritePixel gets)."""
    return g.ctx.render_segment(segment.yBegin, segment.yEnd, segment.xBegin, segment.xEnd, g.g_data, task=False)


def RenderSegmentTask(segment: RenderSegmentData, g: Globals) -> np.ndarray:
    """TaskBasedPathTracer.hpp:54-206 semantics (10-pass cap, count-weighted
    resolve), including the colorIndex stride of non-square tiles (lines 103, 186:
    rows strided by segmentHeight, so pixels alias and some indices stay empty)."""
    return g.ctx.render_segment(segment.yBegin, segment.yEnd, segment.xBegin, segment.xEnd, g.g_data, task=True)


def MakeRenderSegmentData(i, j, segment_width, segment_height, g: Globals) -> RenderSegmentData:
    """Renderer.hpp:232-240."""
    yB = segment_height * j
    yE = g.g_height if yB + segment_height > g.g_height else yB + segment_height
    xB = segment_width * i
    xE = g.g_width if xB + segment_width > g.g_width else xB + segment_width
    return RenderSegmentData(yB, yE, xB, xE)


def RenderImageParallelMain(g: Globals, thread_count: int = 4, task: bool = False) -> None:
    """Renderer.hpp:257-302: a thread_count x thread_count tile grid, at most
    thread_count RenderJob threads in flight, each calling the drop-in entry point
    concurrently on the shared context."""
    tc = thread_count + (thread_count % 2)
    sw, sh = g.g_width // tc, g.g_height // tc
    segments = [MakeRenderSegmentData(i, j, sw, sh, g) for j in range(tc) for i in range(tc)]
    fn = RenderSegmentTask if task else RenderSegment
    errors = []
    sem = threading.Semaphore(tc)

    def job(seg):
        try:
            fn(seg, g)
        except Exception as e:  # surfaced after join
            errors.append(e)
        finally:
            sem.release()

    threads = []
    for seg in segments:
        sem.acquire()
        t = threading.Thread(target=job, args=(seg,))
        t.start()
        threads.append(t)
    for t in threads:
        t.join()
    if errors:
        raise errors[0]


def RenderImage(g: Globals) -> None:
    """Renderer.hpp:304-308: RenderSegmentTask over the full frame."""
    RenderSegmentTask(RenderSegmentData(0, g.g_height, 0, g.g_width), g)
