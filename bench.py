#!/usr/bin/env python3
"""Benchmark of the SimplePathTracer render loop on MI355X.

One step = one frame of BASELINE.json config 2 (GenerateSpheres seed 1,
1200x800, 100 spp, depth 50): every (pixel, sample) path traced by the gfx950
megakernel, folded in sample order, written as float RGBA + RGB8 g_data.
With N GPUs (torchrun, one process per GPU) the frame is split into interleaved
row strips (8 rows, or fewer so the strips deal evenly: 4 at N = 8), rank r renders
strips r, r+N, ...; the float tiles are gathered to rank 0 over RCCL
(all_gather_into_tensor) and assembled there (strong scaling: the frame is fixed,
per-GPU work shrinks with N).  Consecutive frames alternate over two HIP streams
(`--streams`), each with its own workspace and output buffers, so one frame's last
paths drain while the next frame fills the GPU and its gather overlaps rendering.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (scene, width, height, spp, bounces)
    "c2": ("random", 1200, 800, 100, 50),
    "c3": ("random", 3840, 2160, 1024, 50),
    "c5": ("stress10k", 1920, 1080, 256, 50),
    "c1": ("cornell3", 200, 100, 4, 8),
}
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64 T fp32 lane-ops/s (non-FMA)
HBM_PEAK_GBS = 8000.0
FLOP_PER_TEST = 17  # RaySphereIntersection, Collision.hpp:9-17


def make_scene(spt, name):
    if name == "random":
        return spt.generate_spheres(1)
    if name == "stress10k":
        return spt.generate_stress(1, 10000)
    if name == "cornell3":
        return spt.cornell3()
    raise ValueError(name)


def cpu_baseline(scene, view, w, h, spp_sample, bounces, threads):
    """The CPU restatement (oracle/, "port") timed with the reference's
    RenderImageParallelMain tiling (threads x threads tiles, <= threads in
    flight) on RenderSegmentTask, the TaskBasedPathTracer path of north_star."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    osc = pyoracle.OracleScene(scene.centers, scene.radii, scene.colors, scene.materials, scene.fuzz)
    fr = pyoracle.make_frame(view, [0, 1, -3, 0], [137, 207, 240, 0], w, h, spp_sample, bounces, 1)
    t0 = time.perf_counter()
    pyoracle.render_image_parallel(osc, fr, threads, mode=1, want_rgba=False)
    dt = time.perf_counter() - t0
    return {"value": round(w * h * spp_sample / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "kind": "port",
            "sample": f"RenderSegmentTask (oracle C restatement, gcc -O2) via RenderImageParallelMain tiling "
                      f"{threads}x{threads}, same scene/camera at {w}x{h}, {spp_sample} spp, depth {bounces}; "
                      f"{dt:.2f} s wall on {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="segment", choices=["segment", "task"])
    ap.add_argument("--engine", default="megakernel", choices=["megakernel", "wavefront"],
                    help="render loop: persistent megakernel, or the material-queue wavefront variant")
    ap.add_argument("--strip", type=int, default=0, help="rows per strip (0: largest of 8/4/2/1 splitting evenly)")
    ap.add_argument("--streams", type=int, default=0,
                    help="frames in flight on alternating HIP streams (the next frame fills the GPU while "
                         "the previous one's last paths drain; each stream has its own workspace); 0 = auto: "
                         "2 when a frame is one workspace batch, else 1 (long multi-batch frames gain nothing "
                         "and would double the workspace)")
    ap.add_argument("--cpu-spp", type=int, default=32, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump", default="", help="write rank 0's final g_data bytes to this file")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import simplepathtracer_amd as spt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # SPT_DIST_BACKEND=gloo rehearses the N>1 flow with several ranks on one GPU
    backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    scene_name, W, H, spp, bounces = CONFIGS[args.config]
    scene = make_scene(spt, scene_name)
    view = spt.camera_basis()
    mode = spt.MODE_TASK if args.mode == "task" else spt.MODE_SEGMENT
    ctx = spt.Context(local)
    if args.engine == "wavefront":
        ctx.set_engine(spt._native.ENGINE_WAVEFRONT)
    ctx.set_scene(scene)
    ctx.set_camera(view, spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
    ctx.set_params(W, H, spp, bounces, 1)

    from simplepathtracer_amd.distributed import FrameSplit, even_strip, render_frame
    split = FrameSplit(W, H, world, args.strip or even_strip(H, world))
    slot_bytes = 12 if args.mode == "segment" else 16
    one_batch = W * H * spp * slot_bytes <= (16 << 30)  # the context's default workspace
    nst = args.streams if args.streams > 0 else (2 if one_batch else 1)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]
    bufs = []
    for _ in range(nst):  # per-stream frame buffers: frames in flight do not share outputs
        b = {"frame": torch.zeros((H * W, 4), dtype=torch.float32, device=dev) if rank == 0 else None,
             "g_data": torch.zeros(W * H * 3, dtype=torch.uint8, device=dev) if rank == 0 else None,
             "local": None, "gathered": None}
        if world > 1:
            b["local"] = torch.zeros((split.tile_pixels(), 4), dtype=torch.float32, device=dev)
            b["gathered"] = torch.zeros((world * split.tile_pixels(), 4), dtype=torch.float32, device=dev)
        bufs.append(b)
    counter = [0]

    def step():
        k = counter[0] % nst
        counter[0] += 1
        b = bufs[k]
        with torch.cuda.stream(streams[k]):  # RCCL collectives follow the current stream
            render_frame(ctx, split, rank, mode, b["local"], b["gathered"], b["frame"], b["g_data"],
                         streams[k].cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([st["casts"], st["samples"]], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        casts_all, samples_all = float(tot[0]), float(tot[1])
    else:
        casts_all, samples_all = float(st["casts"]), float(st["samples"])

    total_samples = W * H * spp * args.steps
    value = total_samples / elapsed / 1e6
    if rank == 0:
        # dominant kernel = render_kernel; per-launch averages from HIP events on `stream`
        launches = max(st["launches"], 1)
        # per-launch device time = union of the launches' HIP-event intervals / launches:
        # with frames in flight a launch's own span also covers the previous frame's
        # tail (both run at once), so the spans overlap and their sum exceeds the
        # device time; the span average is reported beside it
        avg_ms = st["render_busy_ms"] / launches
        span_ms = st["render_ms"] / launches
        rays_per_launch = st["casts"] / launches
        algo_tflop = FLOP_PER_TEST * scene.n * rays_per_launch / 1e12
        achieved = algo_tflop / (avg_ms / 1e3)
        samples_per_launch = st["samples"] / launches
        slot_bytes = 12.0 if args.mode == "segment" else 16.0  # per-sample slot: rgb (+ counted flag in task mode)
        hbm_bytes = slot_bytes * samples_per_launch  # written by the render kernel
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tpath):
            rec = json.load(open(tpath)).get(args.config, {}).get("render_kernel")
            if rec and world == 1:
                traffic = rec["fetch_bytes"] + rec["write_bytes"]
        out = {
            "metric": "Msamples/s (pixels×spp/s), RTIOW random-sphere scene, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: {scene_name} scene seed 1 (N={scene.n} spheres), {W}x{H}, "
                                   f"{spp} spp, depth {bounces}, {args.mode} mode, {args.engine}",
                       "width": W, "height": H, "spp": spp, "bounces": bounces, "spheres": scene.n,
                       "parallelism": f"row-strips{split.strip}x{world}" if world > 1 else "1 GPU",
                       "frames_in_flight": nst},
            # contract form: the render kernel against HBM (12 B per sample slot written),
            # as BASELINE.json's "fraction of HBM roofline" asks; the kernel is bound by
            # VALU issue and latency instead (roofline_valu)
            "roofline": {"bound": "hbm", "achieved": round(hbm_bytes / (avg_ms / 1e3) / 1e9, 3),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(hbm_bytes / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/traffic.json)",
                         "algorithmic_bytes": hbm_bytes,
                         "kernel": "render_kernel", "avg_launch_ms": round(avg_ms, 4),
                         "avg_launch_ms_def": "union of the render launches' HIP-event intervals (launch stream) / launches",
                         "avg_launch_span_ms": round(span_ms, 4),
                         "binding": "VALU issue + latency (see roofline_valu), not HBM"},
            "roofline_valu": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 2),
                              "unit": "TFLOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
                              "flop_model": "17 FLOP per RaySphereIntersection x N spheres x rays counted in-kernel "
                                            "(brute force; the culling skips most tests, so frac can pass 1)",
                              "rays_per_launch": rays_per_launch,
                              "flop_per_launch": FLOP_PER_TEST * scene.n * rays_per_launch},
            "rays_per_sample": round(casts_all / max(samples_all, 1), 4),
            # with frames in flight the fold runs beside the next frame's render and its
            # own event span mostly measures waiting for CUs: reported for --streams 1 only
            "fold_ms_per_step": round(st["fold_ms"] / args.steps, 4) if nst == 1 else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            cw, ch = (W, H) if args.config != "c3" else (1920, 1080)
            out["cpu_baseline"] = cpu_baseline(scene, view, cw, ch, args.cpu_spp, bounces, args.cpu_threads)
        print(json.dumps(out), flush=True)
        if args.dump:
            torch.cuda.synchronize(dev)
            bufs[(counter[0] - 1) % nst]["g_data"].cpu().numpy().tofile(args.dump)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
