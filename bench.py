#!/usr/bin/env python3
"""Benchmark of the SimplePathTracer render loop on MI355X.

One step = one frame of BASELINE.json config 2 (GenerateSpheres seed 1,
1200x800, 100 spp, depth 50): every (pixel, sample) path traced by the gfx950
megakernel, folded in sample order, written as float RGBA + RGB8 g_data.
With N GPUs (one process per GPU: `--gpus N` starts the N ranks itself when no
launcher did, or torchrun starts them) the frame is split into interleaved
row strips (8 rows, or fewer so the strips deal evenly: 4 at N = 8), rank r renders
strips r, r+N, ...; the float tiles are gathered to rank 0 over RCCL
(one gather: send/recv pairs over xGMI) and assembled there (strong scaling: the frame is fixed,
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
    # BASELINE.json config 2's "~500 spheres": GenerateSpheres' rows run to z < 37.5
    # (488 spheres; the reference's own generator stops at z < 20: 149)
    "c2w": ("random500", 1200, 800, 100, 50),
}
# VALU issue: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles
# (MI355X_MICROARCH.md: 4 SIMD-32 per CU), 1024 SIMDs at 2.4 GHz
CLOCK_HZ = 2.4e9
VALU_ISSUE_PEAK = 256 * 4 * CLOCK_HZ / 2  # 1.2288e12 wave-instructions/s
VALU_PEAK_TOPS = 256 * 4 * 32 * CLOCK_HZ / 1e12  # 78.64 T fp32 lane-ops/s (non-FMA)
HBM_PEAK_GBS = 8000.0
FLOP_PER_TEST = 17  # RaySphereIntersection, Collision.hpp:9-17
VALU_PER_PRETEST = 10  # the conservative member pretest
# algorithmic HBM bytes per frame = 16 B/px float RGBA accumulator + 3 B/px
# RGB8 + 48 B per sphere of scene tables
ALGO_BYTES_PER_PIXEL, ALGO_BYTES_PER_SPHERE = 19, 48
# Reference CPU path vs the restatement, both timed in the build container (8-core Xeon,
# config 2 at 1200x800x100 spp, depth 50, 16 threads = 2*nproc, RenderImageParallelMain
# tiling): reference from BASELINE.md (its clock-seam scene has N = 167), restatement
# measured with `python tools/cpu_calibration.py` (keyed scene seed 1, N = 149)
CPU_CALIBRATION = {"reference_msps": {"segment": 4.26, "task": 4.33},
                   "restatement_msps": {"segment": 5.128, "task": 4.269},
                   "host": "build container, Intel Xeon 8 cores, 16 threads, c2 at 100 spp",
                   "note": "restatement/reference = 1.20 (segment) and 0.99 (task) raw; "
                           "x149/167 sphere-count normalised: 1.07 and 0.88"}


def make_scene(spt, name):
    if name == "random":
        return spt.generate_spheres(1)
    if name == "random500":
        return spt.generate_spheres(1, z_end=37.5)
    if name == "stress10k":
        return spt.generate_stress(1, 10000)
    if name == "cornell3":
        return spt.cornell3()
    raise ValueError(name)


def host_cores():
    """CPUs this process may use: the job's share where one is set (OMP_NUM_THREADS on
    the GPU box, whose os.cpu_count() is the whole machine), else the affinity mask."""
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        return int(share)
    return len(os.sched_getaffinity(0))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def tiled_pixels(w, h, tc):
    """Pixels RenderImageParallelMain actually renders: MakeRenderSegmentData tiles W / tc
    columns and H / tc rows per tile (integer division, Renderer.hpp:264-265), so the
    remainder columns / rows of the frame are never rendered (tc = 32 on 1200 x 800: 1 184
    x 800 pixels)."""
    return (w // tc) * tc * (h // tc) * tc


_T_START = time.perf_counter()


def progress(msg: str) -> None:
    """A progress line on stderr (the JSON line stays the only stdout line): a long
    default run -- CPU baseline, drop-in processes -- keeps showing it is alive."""
    print(f"[bench {time.perf_counter() - _T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(scene, view, w, h, spp_sample, bounces):
    """The CPU restatement (oracle/, "port", gcc -O2 -msse4.1) timed with the
    reference's RenderImageParallelMain tiling (Renderer.hpp:257-302: tc x tc tiles,
    <= tc in flight) at the two thread counts SURVEY §8(d) names: tc = 2 * cores, the
    reference's hardware_concurrency() * 2 rule, and tc = 4, the shipped g_maxThreads
    (Globals.hpp:11; Renderer.hpp:261-262 takes min(2 * hw, g_maxThreads)).
    RenderSegmentTask (TaskBasedPathTracer, north_star's CPU path) at 2 * cores is
    `value`; RenderSegment (the shipped default generation type) beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    osc = pyoracle.OracleScene(scene.centers, scene.radii, scene.colors, scene.materials, scene.fuzz)
    fr = pyoracle.make_frame(view, [0, 1, -3, 0], [137, 207, 240, 0], w, h, spp_sample, bounces, 1)
    cores = host_cores()
    tc = 2 * cores
    res, wall = {}, 0.0
    for threads in (tc, 4):
        for name, mode in (("task", 1), ("segment", 0)):
            t0 = time.perf_counter()
            pyoracle.render_image_parallel(osc, fr, threads, mode=mode, want_rgba=False)
            dt = time.perf_counter() - t0
            progress(f"cpu baseline {name} tc={threads}: {dt:.1f} s")
            wall += dt
            res[(name, threads)] = round(tiled_pixels(w, h, threads) * spp_sample / dt / 1e6, 4)
    return {"value": res[("task", tc)], "unit": "Msamples/s", "cores": cores, "kind": "port",
            "segment_value": res[("segment", tc)], "threads": tc,
            "shipped_tc4": {"task": res[("task", 4)], "segment": res[("segment", 4)],
                            "def": "tc = 4 (g_maxThreads, Globals.hpp:11): 4x4 tiles, <= 4 threads in flight"},
            "nproc": os.cpu_count(), "cpu_model": cpu_model(), "calibration": CPU_CALIBRATION,
            "sample": f"RenderSegmentTask (value) and RenderSegment (segment_value) of the oracle C restatement "
                      f"(gcc -O2 -msse4.1), RenderImageParallelMain tiling {tc}x{tc} with <= {tc} in flight on "
                      f"{cores} cores, and the shipped tc = 4; same scene/camera at {w}x{h}, {spp_sample} spp, "
                      f"depth {bounces}; {wall:.1f} s wall for the four runs; rates count the pixels the tiling "
                      f"renders ((W/tc)*tc x (H/tc)*tc, Renderer.hpp:264-265)"}


def dropin_bench(w, h, spp, bounces, frames, tcs, env=None):
    """The C++ drop-in (include/spt/RenderSegmentShim.hpp) driven exactly like
    RenderImageParallelMain (tools/dropin_harness.cpp): tc x tc RenderJob tiles, <= tc
    threads in flight, host g_data, per tc the Msamples/s of `frames` timed frames; and
    the calling pattern's own ceiling: the same frames with RenderJob doing nothing
    (SPT_HARNESS_NOOP), as ms per frame and the rate it would allow."""
    import subprocess
    exe = os.path.join(ROOT, "simplepathtracer_amd", "lib", "spt_dropin_harness")
    if not os.path.exists(exe):
        return None
    out = {}
    run_env = dict(os.environ, **(env or {}))

    def harness(args, extra_env, what):
        # bounded: a harness that does not finish is reported in the line, not waited for
        # (the bench line must still print)
        progress(f"drop-in {what} ...")
        try:
            return subprocess.run([exe, "/dev/null", *map(str, args)], capture_output=True, text=True, timeout=90,
                                  env=dict(run_env, **extra_env))
        except subprocess.TimeoutExpired:
            out.setdefault("errors", []).append(f"{what}: no result within 90 s")
            progress(f"drop-in {what}: timed out")
            return None

    # the reference app's own pattern (Renderer.hpp:335-344 MainLoop renders one frame per
    # process): a fresh process per run, its one frame timed in parts (median of 3 runs)
    for task in (0, 1):
        tc = 4
        runs = []
        for _ in range(3):
            r = harness((w, h, spp, bounces, tc, task, 0), {"SPT_HARNESS_COLD": "1"}, f"cold task={task} tc={tc}")
            if r is None:
                continue
            if r.returncode != 0:
                out.setdefault("errors", []).append(f"cold task={task}: rc {r.returncode}: {r.stderr[-300:]}")
                continue
            line = r.stdout.split("cold ", 1)[1].split("\n")[0]
            progress(f"drop-in cold {'task' if task else 'segment'} tc={tc}: {line}")
            runs.append({k: float(v) for k, v in (kv.split("=") for kv in line.split())})
        if not runs:
            continue
        med = {k: float(np.median([x[k] for x in runs])) for k in ("ctx_ms", "setup_ms", "frame_ms", "accel_ms", "prim_ms")}
        key = f"cold_{'task' if task else 'segment'}_tc{tc}"
        out[key] = {k: round(v, 3) for k, v in med.items()}
        out[key]["total_ms"] = round(med["ctx_ms"] + med["setup_ms"] + med["frame_ms"], 3)
        out[key]["frame_msamples_s"] = round(tiled_pixels(w, h, tc) * spp / med["frame_ms"] / 1e3, 1)
    for tc in tcs:
        r = harness((w, h, spp, bounces, tc, 0, frames), {"SPT_HARNESS_NOOP": "1"}, f"noop tc={tc}")
        if r is not None and r.returncode == 0:
            sec = float(r.stdout.split("seconds=")[1].split()[0])
            out[f"noop_tc{tc}_ms_per_frame"] = round(sec / frames * 1e3, 3)
            out[f"noop_tc{tc}_ceiling"] = round(tiled_pixels(w, h, tc) * spp * frames / sec / 1e6, 1)
        for task in (0, 1):
            r = harness((w, h, spp, bounces, tc, task, frames), {}, f"repeated task={task} tc={tc}")
            if r is None:
                continue
            if r.returncode != 0:
                out.setdefault("errors", []).append(f"repeated task={task} tc={tc}: rc {r.returncode}: {r.stderr[-300:]}")
                continue
            sec = float(r.stdout.split("seconds=")[1].split()[0])
            key = f"{'task' if task else 'segment'}_tc{tc}"
            progress(f"drop-in {key}: {frames} frames in {sec:.2f} s")
            out[key] = round(tiled_pixels(w, h, tc) * spp * frames / sec / 1e6, 3)
            if "batches=" in r.stdout:  # calls per batched launch, over all frames run
                calls = int(r.stdout.split("calls=")[1].split()[0])
                batches = int(r.stdout.split("batches=")[1].split()[0])
                out[key + "_calls_per_batch"] = round(calls / max(batches, 1), 2)
    return out


def profile_record(config):
    """Per-launch PMC counters and in-kernel lane counts of the render kernel for a
    config, from profiles/counters.json (rocprofv3 --pmc passes and the SPT_DIAG build,
    tools/profile.sh + tools/summarize_profile.py), or None."""
    path = os.path.join(ROOT, "profiles", "counters.json")
    if not os.path.exists(path):
        return None
    return json.load(open(path)).get(config)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) run without a launcher: start the N rank processes as children
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) and return
    their exit code.  Nothing here touches the GPU (counting devices does not initialise
    HIP on this image), so no process that initialised the GPU ever execs.  The GPU
    count is checked first: N ranks over RCCL need N visible GPUs, and the run is
    refused (exit 2) rather than silently rendering on fewer; SPT_DIST_BACKEND=gloo is
    the rehearsal backend, whose ranks may share a GPU (rank r uses GPU r % count)."""
    import subprocess
    import torch
    backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
    have = torch.cuda.device_count()
    if not args.launch_check and backend == "nccl" and args.gpus > have:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {have} visible", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def launch_check(args) -> None:
    """--launch-check: each rank joins the process group (SPT_DIST_BACKEND, gloo on a
    CPU-only host) and rank 0 prints what the group sees; no GPU work."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("SPT_DIST_BACKEND", "gloo")
    if world > 1:
        dist.init_process_group(backend)
        ids = torch.zeros((world, 2), dtype=torch.int64)
        ids[rank] = torch.tensor([rank, local])
        dist.all_reduce(ids)
        seen = {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": ids[:, 0].tolist(),
                "local_ranks": ids[:, 1].tolist()}
        dist.destroy_process_group()
    else:
        seen = {"world_size": 1, "backend": None, "ranks": [0], "local_ranks": [0]}
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": args.gpus, **seen}), flush=True)


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
    ap.add_argument("--service", type=int, default=-1,
                    help="1: frames are jobs of the resident render service (spt_service_start: one persistent "
                         "launch per timed region, no launch ramp and tail per frame); 0: one launch per frame; "
                         "-1 (default): the service for the rank shares of N > 1 ranks, launches at N = 1 "
                         "(profiles/svc_timeline_r04.txt: 20 config-2 frames, 1/8 shares 13.4 vs 14.4 ms, "
                         "whole frames 95.0 vs 92.9 ms)")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "ipc"],
                    help="N > 1: how the rank tiles reach rank 0: the copy-engine transport (distributed."
                         "TileTransport: peer copies from IPC handles ordered by stream wait/write-value packets, "
                         "no collective kernel; the session keeps one block slot per CU free for the folds and "
                         "assembles: DESIGN.md §5 Round 6) when its setup check passes on every rank, else one "
                         "RCCL gather per frame (auto, default); rccl / ipc force one (ipc: exit if the check "
                         "fails)")
    ap.add_argument("--cpu-spp", type=int, default=0,
                    help="spp of the CPU-baseline sample (0: the config's own spp on config 2, scaled down on others)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the C++ drop-in measurement (config 2)")
    ap.add_argument("--dropin-frames", type=int, default=20)
    ap.add_argument("--dump", default="", help="write rank 0's final g_data bytes to this file")
    ap.add_argument("--launch-check", action="store_true",
                    help="only start the ranks and report the process group (launcher test; no GPU work)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args, sys.argv[1:]))
    if args.launch_check:
        launch_check(args)
        return

    import torch
    import torch.distributed as dist
    import simplepathtracer_amd as spt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # SPT_DIST_BACKEND=gloo rehearses the N>1 flow with several ranks on one GPU
    backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks over RCCL need {world} GPUs, {ndev} visible")
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    # the render service (--service 1) is started around each timed region and stopped
    # (drained) inside it: a device-wide synchronisation must not wait for its resident kernel
    # (auto: rank shares of N > 1 ranks, each on a GPU of its own -- ranks rehearsed on a
    # shared GPU would hold each other's resident kernels off the CUs).  With the RCCL gather
    # the session takes every block slot (spt_service_set_full_grid): RCCL's kernel needs a
    # whole CU, so the folds and gathers of a region's frames run after its session ends
    # anyway (N = 8 shares with a gather stand-in: 0.740 vs 0.756 ms per share; DESIGN.md
    # §5); with the copy-engine transport one slot per CU stays free for the folds, wait
    # packets and assembles, which then overlap the session (0.847 vs 0.757 in the one-GPU
    # rehearsal, profiles/scaling_r06.txt)
    auto_svc = world > 1 and world <= torch.cuda.device_count()
    use_svc = (args.service if args.service >= 0 else auto_svc) and args.engine == "megakernel"
    try_ipc = world > 1 and args.transport in ("auto", "ipc")
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
    slot_bytes = 4 if args.mode == "segment" else 8  # sample words (+ the order key in task mode)
    one_batch = W * H * spp * slot_bytes <= (16 << 30)  # the context's default workspace
    nst = args.streams
    if nst <= 0:
        # two frames in flight when a frame is one sample batch (the next frame's blocks
        # take the CUs as this one's drain; config 2: 22 849-22 878 vs 3 streams 22 685-
        # 22 728; config 5's 1024-thread LDS-tree blocks: 7 478-7 495 vs one stream
        # 7 459-7 474 on the round-5 kernels); several sample batches
        # (config 3) overlap through their own companion stream
        nst = 2 if one_batch else 1
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]
    bufs = []
    for _ in range(nst):  # per-stream frame buffers: frames in flight do not share outputs
        b = {"frame": torch.zeros((H * W, 4), dtype=torch.float32, device=dev) if rank == 0 else None,
             "g_data": torch.zeros(W * H * 3, dtype=torch.uint8, device=dev) if rank == 0 else None,
             "local": None, "gathered": None}
        if world > 1:
            b["local"] = torch.zeros((split.slot_pixels(mode), 4), dtype=torch.float32, device=dev)
        bufs.append(b)
    transport, transport_check = None, None
    if try_ipc:
        from simplepathtracer_amd.distributed import TileTransport
        # one gathered buffer per stream: frames f and f + nst share a stream (step below);
        # kept only if its setup check passes on every rank (else the RCCL gather)
        try:
            transport = TileTransport(ctx, split, rank, nbuf=nst, mode=mode)
            ok = transport.verify(bufs[0]["local"], streams[0])
        except RuntimeError as e:  # the setup failed on some rank: every rank raises it
            progress(f"rank {rank}: copy-engine transport setup failed: {e}")
            transport, ok = None, False
        transport_check = "passed" if ok else "failed"
        if not ok:
            if transport is not None:
                transport.close()
            transport = None
            if args.transport == "ipc":
                raise SystemExit("bench.py: --transport ipc: the transport's setup check failed")
        progress(f"rank {rank}: tile transport {'copy-engine (IPC)' if transport else 'RCCL gather'}")
    if world > 1 and rank == 0 and transport is None:
        for b in bufs:
            b["gathered"] = torch.zeros((world * split.slot_pixels(mode), 4), dtype=torch.float32, device=dev)
    if use_svc and "SPT_SVC_FULL_GRID" not in os.environ:
        ctx.service_set_full_grid(transport is None)
    counter = [0]
    # gather timing of the timed steps (N > 1): events around each step's gather
    gev = []

    def step(timed=False):
        f = counter[0]
        k = f % nst
        counter[0] += 1
        b = bufs[k]
        ev = None
        if timed and world > 1:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            gev.append(ev)
        with torch.cuda.stream(streams[k]):  # RCCL collectives follow the current stream
            render_frame(ctx, split, rank, mode, b["local"], b["gathered"], b["frame"], b["g_data"],
                         streams[k].cuda_stream, gather_events=ev, transport=transport, frame_no=f)

    progress(f"rank {rank}: {args.config} ready (setup {ctx.stats()['prim_list_build_ms']:.1f} ms of lists), "
             f"{args.warmup} warm-up steps")
    if use_svc:
        ctx.service_start()
    for _ in range(args.warmup):
        step()
    if use_svc:
        ctx.service_stop()
    torch.cuda.synchronize(dev)
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    progress(f"rank {rank}: warm-up done, timing {args.steps} steps")
    t0 = time.perf_counter()
    if use_svc:
        ctx.service_start()
    for _ in range(args.steps):
        step(timed=True)
    if use_svc:
        ctx.service_stop()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    # this rank's render device time per step (union of its launches' intervals; the
    # render service: its session kernel's time)
    rank_render_ms = (st["svc_kernel_ms"] if use_svc else st["render_busy_ms"]) / args.steps
    rank_gather_ms = sum(a.elapsed_time(b) for a, b in gev) / max(len(gev), 1)
    per_rank = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([st["casts"], st["samples"]], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        casts_all, samples_all = float(tot[0]), float(tot[1])
        pr = torch.zeros((2, world), dtype=torch.float64, device=dev)
        pr[0, rank] = rank_render_ms
        pr[1, rank] = rank_gather_ms
        dist.all_reduce(pr)
        per_rank = pr.cpu().tolist()
        world_seen, backend_seen = dist.get_world_size(), dist.get_backend()
    else:
        casts_all, samples_all = float(st["casts"]), float(st["samples"])
        world_seen, backend_seen = 1, None

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
        if use_svc:
            # the render service: one resident launch per timed region, one job per frame;
            # the per-frame device time is the session kernel's time over its jobs
            launches = max(st["svc_jobs"], 1)
            avg_ms = span_ms = st["svc_kernel_ms"] / launches
        t_launch = avg_ms / 1e3
        rays_per_launch = st["casts"] / launches
        samples_per_launch = st["samples"] / launches
        px_per_launch = samples_per_launch / spp  # every launch renders its pixels at full spp
        # SURVEY §8(d) algorithmic bytes: 19 B per pixel (float RGBA + RGB8) + 48 B per sphere
        algo_bytes = ALGO_BYTES_PER_PIXEL * px_per_launch + ALGO_BYTES_PER_SPHERE * scene.n
        slot_bytes = (4.0 if args.mode == "segment" else 8.0) * samples_per_launch  # the design's sample slots
        prof = profile_record(args.config) if world == 1 and args.engine == "megakernel" else None
        rk = (prof or {}).get("render_kernel", {})
        fk = (prof or {}).get("fold_kernel", {})
        traffic = (rk["fetch_bytes"] + rk["write_bytes"]) if "fetch_bytes" in rk else None
        frame_traffic = traffic + fk["fetch_bytes"] + fk["write_bytes"] if traffic and "fetch_bytes" in fk else None
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
                       "frames_in_flight": nst, "render_service": bool(use_svc),
                       "transport": (("ipc" if transport is not None else "rccl") if world > 1 else None),
                       "transport_check": transport_check,
                       "service_full_grid": bool(use_svc) and (os.environ.get("SPT_SVC_FULL_GRID", "0") != "0"
                                                               if "SPT_SVC_FULL_GRID" in os.environ
                                                               else transport is None)},
            # contract form: the render kernel against HBM with SURVEY §8(d)'s algorithmic
            # bytes; HBM does not bind this kernel (VALU issue + latency do: roofline_valu)
            "roofline": {"bound": "hbm", "achieved": round(algo_bytes / t_launch / 1e9, 4),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo_bytes / t_launch / 1e9 / HBM_PEAK_GBS, 7), "traffic": traffic,
                         "traffic_unit": "HBM bytes per render launch (PMC FETCH_SIZE x2 + WRITE_SIZE, "
                                         "profiles/counters.json)",
                         "algorithmic_bytes": algo_bytes,
                         "algorithmic_def": "19 B x pixels + 48 B x spheres per launch (SURVEY §8d)",
                         "traffic_over_algorithmic": round(traffic / algo_bytes, 1) if traffic else None,
                         "render_write_over_slots": round(rk["write_bytes"] / slot_bytes, 3) if traffic else None,
                         "frame_traffic": frame_traffic,
                         "frame_traffic_def": "render FETCH x2 + WRITE plus the fold's FETCH x2 + WRITE per launch "
                                              "(PMC, profiles/counters.json)",
                         "frame_traffic_over_algorithmic": round(frame_traffic / algo_bytes, 1) if frame_traffic
                                                           else None,
                         "slot_bytes": slot_bytes,
                         "slot_def": "the design's per-sample slots (a 4-byte sample word in segment mode, word + "
                                     "order key in task mode) written once by the render kernel and read back "
                                     "once by the fold",
                         "kernel": "render_kernel_svc" if use_svc else "render_kernel",
                         "avg_launch_ms": round(avg_ms, 4),
                         "avg_launch_ms_def": ("the session kernel's HIP-event interval / its jobs (one per frame)"
                                               if use_svc else "union of the render launches' HIP-event intervals "
                                                               "(launch stream) / launches"),
                         "avg_launch_span_ms": round(span_ms, 4)},
            "world_size": world_seen,
            "backend": backend_seen,
            "rays_per_sample": round(casts_all / max(samples_all, 1), 4),
            # host setup outside the timed region, once per scene / camera / frame size: the
            # traversal tables (build, check, upload) and the primary-ray candidate lists
            "setup_ms": {"accel_build_ms": round(st["accel_build_ms"], 3),
                         "prim_list_build_ms": round(st["prim_list_build_ms"], 3),
                         "total_ms": round(st["accel_build_ms"] + st["prim_list_build_ms"], 3)},
            # a fold overlapped by another stream's render (frames in flight, or the double-buffered
            # sample batches of a multi-batch frame) spans its wait for free CU slots: not reported
            "fold_ms_per_step": round(st["fold_ms"] / args.steps, 4) if nst == 1 and one_batch else None,
        }
        if per_rank is not None:
            out["ranks"] = {"render_ms": [round(v, 4) for v in per_rank[0]],
                            "gather_ms": [round(v, 4) for v in per_rank[1]],
                            "def": "per rank and step: render device time (union of its render launches' HIP-event "
                                   "intervals) and the gather (HIP events on the step's stream around dist.gather, "
                                   "or around the transport's send / receive packets; includes waiting for the "
                                   "slowest rank)"}
        if prof and "SQ_INSTS_VALU" in rk:
            # the binding resource: VALU issue.  Wave-instructions per launch from the PMC
            # pass over this same command, against 1024 SIMDs x 2.4 GHz / 2 cycles per
            # wave64 instruction; lane-level work from the SPT_DIAG build's in-kernel counts
            issue = rk["SQ_INSTS_VALU"] / t_launch
            rv = {"bound": "valu-issue", "achieved": round(issue / 1e12, 5), "peak": round(VALU_ISSUE_PEAK / 1e12, 5),
                  "unit": "T wave64-VALU-instructions/s", "frac": round(issue / VALU_ISSUE_PEAK, 4),
                  "valu_insts_per_launch": rk["SQ_INSTS_VALU"], "salu_insts_per_launch": rk.get("SQ_INSTS_SALU"),
                  "source": rk.get("source")}
            dg = (prof or {}).get("diag")
            if dg:
                lane_ops = (FLOP_PER_TEST * dg["lane_tests_per_ray"] + VALU_PER_PRETEST * dg["lane_pretests_per_ray"]) \
                    * rays_per_launch
                rv["useful"] = {"achieved": round(lane_ops / t_launch / 1e12, 3), "peak": round(VALU_PEAK_TOPS, 2),
                                "unit": "T fp32 lane-ops/s", "frac": round(lane_ops / t_launch / 1e12 / VALU_PEAK_TOPS, 4),
                                "tests_per_ray": dg["lane_tests_per_ray"],
                                "pretests_per_ray": dg["lane_pretests_per_ray"],
                                "brute_force_tests_per_ray": scene.n,
                                "def": "17 FLOP per RaySphereIntersection + 10 per member pretest, evaluated for "
                                       "live lanes (SPT_DIAG in-kernel counts, profiles/counters.json) x rays "
                                       "counted in-kernel / launch time"}
            # VALUUtilization: active lanes per VALU instruction (%); occupancy: mean resident
            # waves per SIMD over the launch (MeanOccupancyPerCU / 4); scalar-cache miss rate
            for k in ("VALUUtilization", "occupancy_waves_per_simd", "sqc_dcache_miss_frac"):
                if k in rk:
                    rv[k] = rk[k]
            out["roofline_valu"] = rv
        if world == 1 and not args.no_cpu_baseline:
            # config 2 at its own 100 spp; the larger configs at their scene and depth, on
            # config 2's frame, with spp scaled down to a bounded sample (c5's 10 000
            # spheres are scanned brute force by the reference's loop)
            cpu_spp = args.cpu_spp or (spp if args.config == "c2" else max(1, round(100 * 149 / scene.n)))
            cw, ch = (W, H) if args.config in ("c1", "c2") else (1200, 800)
            progress("timed region done; CPU baseline")
            out["cpu_baseline"] = cpu_baseline(scene, view, cw, ch, cpu_spp, bounces)
        if world == 1 and args.config == "c2" and not args.no_dropin and args.engine == "megakernel":
            # the drop-in boundary itself: RenderSegment/RenderSegmentTask from RenderJob threads
            progress("C++ drop-in legs")
            try:
                d = dropin_bench(W, H, spp, bounces, args.dropin_frames, (4, 2 * host_cores()))
            except Exception as e:  # the measured line prints whatever a side leg does
                d = {"errors": [f"{type(e).__name__}: {e}"[:400]]}
            if d:
                out["dropin"] = {"unit": "Msamples/s", **d,
                                 "def": "C++ shim under RenderImageParallelMain tiling (tools/dropin_harness.cpp), "
                                        "host g_data, tc=4 (shipped g_maxThreads) and tc=2*cores; rates count the "
                                        "pixels the tiling renders ((W/tc)*tc x (H/tc)*tc, Renderer.hpp:264-265). "
                                        "cold_*: what the reference app gets -- MainLoop renders ONE frame per "
                                        "process (Renderer.hpp:335-344): a fresh process, context creation, the "
                                        "globals' upload (scene, traversal tables, primary-ray lists, g_data "
                                        "page-locking) and that one frame, each timed (median of 3 processes). "
                                        f"segment_tc*/task_tc*: REPEATED frames, {args.dropin_frames} timed after "
                                        "an untimed one; a pattern the reference app never produces, served by "
                                        "the shim's tiling read-ahead (spt_batch.cpp SpecFrame: once a tiling has "
                                        "been called whole, the whole frame renders in 4 launches at its next "
                                        "first tile; SPT_READAHEAD=0 turns it off)"}
        print(json.dumps(out), flush=True)
        if args.dump:
            torch.cuda.synchronize(dev)
            bufs[(counter[0] - 1) % nst]["g_data"].cpu().numpy().tofile(args.dump)
    if transport is not None:
        transport.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
