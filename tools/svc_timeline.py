"""Per-frame completion times of one timed region (service on/off): an event after each
frame's fold on its stream; prints the completion times relative to the region's start,
the steady-state slope (least squares over frames 2..K-1) and the intercept.
Usage (GPU box): python tools/svc_timeline.py [--n 8] [--frames 20] [--service 1]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402
from simplepathtracer_amd.distributed import FrameSplit, even_strip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--service", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
W, H, SPP, B = 1200, 800, 100, 50
ctx = spt.Context(0)
ctx.set_scene(spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, SPP, B, 1)
n = args.n
split = FrameSplit(W, H, n, even_strip(H, n))
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
tiles = [torch.zeros((split.tile_pixels(), 4), dtype=torch.float32, device="cuda") for _ in streams]
torch.cuda.synchronize()
for r in range(args.reps + 1):
    ctx.synchronize()
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    start.record(streams[0])
    streams[1].wait_stream(streams[0])
    t0 = time.perf_counter()
    if args.service:
        ctx.service_start()
    t_svc = (time.perf_counter() - t0) * 1e3  # host time of service_start
    evs = []
    for k in range(args.frames):
        st = streams[k % 2]
        ctx.render_rows_async(spt.MODE_SEGMENT, 0, H, split.strip if n > 1 else 1, n, 0, 0, W,
                              tiles[k % 2].data_ptr(), 0, st.cuda_stream)
        e = torch.cuda.Event(enable_timing=True)
        e.record(st)
        evs.append(e)
        if k == 0:
            t_first = (time.perf_counter() - t0) * 1e3
    t_enq = (time.perf_counter() - t0) * 1e3
    if args.service:
        ctx.service_stop()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    ts = np.array([start.elapsed_time(e) for e in evs])
    if r == 0:
        continue
    k = np.arange(len(ts))
    sl, ic = np.polyfit(k[2:-1], ts[2:-1], 1)
    print(f"rep {r}: N={n} service={args.service} host: start {t_svc:.3f}, first job {t_first:.3f}, "
          f"enqueue {t_enq:.2f} ms, wall {wall:.2f} ms, "
          f"frames done at {' '.join(f'{x:.2f}' for x in ts)} ms; slope {sl:.4f} ms/frame, intercept {ic:.3f} ms",
          flush=True)
ctx.close()
