"""Strong-scaling probe on ONE GPU: device time of the render kernel for the rows
one rank of an N-rank job owns (interleaved 8-row strips), vs the full frame.
Usage (GPU box): python tools/scaling_probe.py [--config c2] [--reps 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402
from simplepathtracer_amd.distributed import FrameSplit, even_strip  # noqa: E402
import time  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--streams", type=int, default=1, help="frames in flight on alternating streams (wall time)")
ap.add_argument("--frames", type=int, default=8)
args = ap.parse_args()
W, H, SPP, B = {"c2": (1200, 800, 100, 50), "c3": (3840, 2160, 1024, 50)}[args.config]
ctx = spt.Context(0)
ctx.set_scene(spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, SPP, B, 1)
base = None
streams = [torch.cuda.Stream() for _ in range(args.streams)]
for n in (1, 2, 4, 8):
    split = FrameSplit(W, H, n, even_strip(H, n))
    tiles = [torch.zeros((split.tile_pixels(), 4), dtype=torch.float32, device="cuda") for _ in streams]

    def frame(k):
        ctx.render_rows_async(spt.MODE_SEGMENT, 0, H, split.strip if n > 1 else 1, n, 0, 0, W,
                              tiles[k % len(streams)].data_ptr(), 0, streams[k % len(streams)].cuda_stream)

    ts = []
    for r in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.frames):
            frame(k)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3 / args.frames)
    t = float(np.median(ts))
    base = base or t
    print(f"N={n}: rank-0 share {split.rows[0]} rows (strip {split.strip}), wall per frame {t:8.3f} ms "
          f"({args.streams} stream(s)), ideal {base / n:8.3f} ms, efficiency {base / n / t:6.3f}", flush=True)
