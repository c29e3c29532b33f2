"""simplepathtracer_amd -- MI355X-native render loop of SimplePathTracer.

The per-pixel render loop (RenderSegment / RenderSegmentTask ->
TraceAndSampleColor -> SampleColor* -> FindClosestIntersectionSphere) runs as
hand-written HIP kernels for gfx950 behind the C ABI in include/spt_hip.h.
"""
from ._native import MODE_SEGMENT, MODE_TASK, SptError, build, lib  # noqa: F401
from .scene import (DIFFUSE, REFLECTIVE, REFRACTIVE, SKYBOX, INIT_COLOR, Scene, camera_basis, cornell3,  # noqa: F401
                    generate_spheres, generate_stress, init_spheres)
from .renderer import (Context, Globals, MakeRenderSegmentData, RenderImage, RenderImageParallelMain,  # noqa: F401
                       RenderSegment, RenderSegmentData, RenderSegmentTask, SaveImage, rows_count)

__all__ = [
    "SaveImage", "MODE_SEGMENT", "MODE_TASK", "SptError", "build", "lib", "Scene", "camera_basis", "cornell3",
    "generate_spheres", "generate_stress", "init_spheres", "Context", "Globals", "MakeRenderSegmentData",
    "RenderImage", "RenderImageParallelMain", "RenderSegment", "RenderSegmentData", "RenderSegmentTask",
    "rows_count", "DIFFUSE", "REFLECTIVE", "REFRACTIVE", "SKYBOX", "INIT_COLOR",
]
