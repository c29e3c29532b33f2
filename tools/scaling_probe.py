"""Strong-scaling probe on ONE GPU: wall time per frame of the rows one rank of an N-rank
job owns (interleaved strips, the bench's split) against the full frame, with frames in
flight on alternating streams, through the render service (--service 1) or one launch
per frame (--service 0).  Per-rank efficiency = (full-frame time / N) / share time.
--record FILE writes the table with its settings and the build it ran (one record per
build and setting: profiles/scaling_<round>.txt keeps them).
Usage (GPU box): python tools/scaling_probe.py [--config c2] [--reps 5] [--streams 2] [--service 1]"""
import argparse
import datetime
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402
from simplepathtracer_amd.distributed import FrameSplit, even_strip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--streams", type=int, default=1, help="frames in flight on alternating streams (wall time)")
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--service", type=int, default=1)
ap.add_argument("--record", default="")
ap.add_argument("--ns", default="1,2,4,8", help="rank counts to probe")
ap.add_argument("--stats", type=int, default=0, help="print the context's service counters per N")
ap.add_argument("--strip", type=int, default=0, help="rows per interleaved strip (0: even_strip, the bench's)")
ap.add_argument("--reserve", type=int, default=0, help="CUs kept free of launched renders (spt_set_reserved_cus)")
ap.add_argument("--blocker", type=int, default=0,
                help="after each frame, a collective stand-in of this many us (tests/cpp/spt_testhooks.hip's "
                     "blocker: 8 blocks of 256-VGPR waves, like RCCL's gather kernel) on a third stream")
ap.add_argument("--sdma", type=int, default=0,
                help="after each frame, copy its tile to page-locked host memory on a third stream (a copy-engine "
                     "transfer that needs no CU: the stand-in for a peer copy over xGMI); the frame after next waits")
args = ap.parse_args()
W, H, SPP, B = {"c2": (1200, 800, 100, 50), "c3": (3840, 2160, 1024, 50), "c5": (1920, 1080, 256, 50)}[args.config]
ctx = spt.Context(0)
# config 5: the 10 000-sphere stress scene (bench.py make_scene "stress10k"; LDS lane walk)
ctx.set_scene(spt.generate_stress(1, 10000) if args.config == "c5" else spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, SPP, B, 1)
ctx.set_reserved_cus(args.reserve)
base = None
streams = [torch.cuda.Stream() for _ in range(args.streams)]
comm = torch.cuda.Stream()
if args.blocker:
    import ctypes
    hooks = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simplepathtracer_amd",
                                     "lib", "libspt_testhooks.so"))
    hooks.spt_test_blocker.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
lines = []
for n in [int(x) for x in args.ns.split(",")]:
    split = FrameSplit(W, H, n, args.strip or even_strip(H, n))
    tiles = [torch.zeros((split.tile_pixels(), 4), dtype=torch.float32, device="cuda") for _ in streams]
    hosts = [torch.zeros((split.tile_pixels(), 4), dtype=torch.float32).pin_memory() for _ in streams] if args.sdma else []

    def frame(k):
        ctx.render_rows_async(spt.MODE_SEGMENT, 0, H, split.strip if n > 1 else 1, n, 0, 0, W,
                              tiles[k % len(streams)].data_ptr(), 0, streams[k % len(streams)].cuda_stream)
        if args.blocker:
            # the frame's gather: on the comm stream once the frame is done; the next frame
            # on the render stream waits for it (the bench's tile buffer reuse)
            s = streams[k % len(streams)]
            comm.wait_stream(s)
            assert hooks.spt_test_blocker(ctypes.c_void_p(comm.cuda_stream), args.blocker, 8, None) == 0
            s.wait_stream(comm)
        if args.sdma:
            s = streams[k % len(streams)]
            comm.wait_stream(s)
            with torch.cuda.stream(comm):
                hosts[k % len(streams)].copy_(tiles[k % len(streams)], non_blocking=True)
            s.wait_stream(comm)

    ts = []
    ctx.reset_stats()
    for r in range(args.reps + 1):
        ctx.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if args.service:
            ctx.service_start()
        for k in range(args.frames):
            frame(k)
        if args.service:
            ctx.service_stop()
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3 / args.frames)
    t = float(np.median(ts))
    base = base or t
    line = (f"N={n}: rank-0 share {split.rows[0]} rows (strip {split.strip}), wall per frame {t:8.3f} ms "
            f"({args.streams} stream(s)), ideal {base / n:8.3f} ms, efficiency {base / n / t:6.3f}")
    print(line, flush=True)
    lines.append(line)
    if args.stats:
        st = ctx.stats()
        print("   stats: " + " ".join(f"{k}={st[k]}" for k in ("launches", "svc_sessions", "svc_jobs", "svc_watchdog_exits",
                                                               "svc_kernel_ms", "svc_grid_blocks", "render_busy_ms")),
              flush=True)
if args.record:
    try:
        head = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip() or "unknown"
    except OSError:
        head = "unknown"
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simplepathtracer_amd", "lib",
                      "libspt_hip.so")
    with open(args.record, "w") as f:
        f.write(f"# tools/scaling_probe.py --config {args.config} --streams {args.streams} --frames {args.frames} "
                f"--reps {args.reps} --service {args.service} --reserve {args.reserve} --blocker {args.blocker} "
                f"--sdma {args.sdma}\n")
        f.write(f"# {datetime.datetime.now().isoformat(timespec='seconds')}, git {head}, libspt_hip.so mtime "
                f"{datetime.datetime.fromtimestamp(os.path.getmtime(so)).isoformat(timespec='seconds')}, "
                f"env SPT_*: {' '.join(f'{k}={v}' for k, v in sorted(os.environ.items()) if k.startswith('SPT_')) or '-'}\n")
        f.write("# wall time per frame over the frames of one timed region (median of reps); the frame's "
                "rows as one rank of N owns them, on one GPU\n")
        f.write("\n".join(lines) + "\n")
ctx.close()
