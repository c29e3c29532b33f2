"""GPU tests of the resident render service (spt_service_start, DESIGN.md §5 "Render
service"): frames, rank shares, sample batches and task-mode jobs rendered as jobs of
one persistent launch must be bit-identical to the launched renders (and those are
pinned against the oracle by test_gpu_parity.py), and every session must end cleanly.
Every device synchronisation here goes through ctx.service_stop()/ctx.synchronize()
first (a device-wide sync would wait for the resident kernel to idle out)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EYE, LOOK, UP, SKY = [0, 1, -3, 0], [0, 1, 0, 0], [0, 1, 0, 0], [137, 207, 240, 0]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_bitwise(got, want, what=""):
    g, w = bits(got), bits(want)
    bad = np.nonzero(g != w)
    assert not len(bad[0]), f"{what}: {len(bad[0])} of {g.size} lanes differ"


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


def make_ctx(spt, golden_scenes, w, h, spp, bounces, seed=1, name="random"):
    gs = golden_scenes
    c = spt.Context(0)
    c.set_scene(spt.Scene(*(gs[f"{name}_{k}"] for k in ("centers", "radii", "colors", "materials", "fuzz"))))
    c.set_camera(spt.camera_basis(EYE, LOOK, UP), EYE, SKY)
    c.set_params(w, h, spp, bounces, seed)
    return c


def render_frames(ctx, jobs, W, H, mode, streams, service):
    """jobs: list of (yB, yE, strip, parts, part, xB, xE); each rendered into its own
    device buffers on alternating streams, all enqueued before any synchronisation."""
    import torch
    from simplepathtracer_amd.renderer import rows_count
    outs = []
    for yB, yE, strip, parts, part, xB, xE in jobs:
        n = rows_count(yB, yE, strip, parts, part) * (xE - xB)
        outs.append((torch.zeros((max(n, 1), 4), dtype=torch.float32, device="cuda"),
                     torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")))
    # the zero fills run on torch's current stream: done before any render stream writes
    torch.cuda.synchronize()
    if service:
        ctx.service_start()
    for k, (yB, yE, strip, parts, part, xB, xE) in enumerate(jobs):
        rgba, g8 = outs[k]
        st = streams[k % len(streams)]
        ctx.render_rows_async(mode, yB, yE, strip, parts, part, xB, xE, rgba.data_ptr(), g8.data_ptr(), st.cuda_stream)
    if service:
        ctx.service_stop()
    ctx.synchronize()
    torch.cuda.synchronize()
    return [(a.cpu().numpy(), b.cpu().numpy()) for a, b in outs]


@pytest.mark.parametrize("full", [0, 1])
@pytest.mark.parametrize("mode", [0, 1])
def test_service_frames_equal_launched_frames(spt, golden_scenes, monkeypatch, mode, full):
    """K consecutive frames through the queue, each compared with a one-shot render; also
    with the session on every block slot (SPT_SVC_FULL_GRID, bench.py's N > 1 regions),
    whose fold launches on the caller's streams then run after the session ends."""
    import torch
    monkeypatch.setenv("SPT_SVC_FULL_GRID", str(full))
    W, H = 320, 200
    ctx = make_ctx(spt, golden_scenes, W, H, 16, 50, seed=3)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = [(0, H, 1, 1, 0, 0, W)] * 5
    ref = render_frames(ctx, jobs[:1], W, H, mode, streams, service=False)[0]
    ctx.reset_stats()
    got = render_frames(ctx, jobs, W, H, mode, streams, service=True)
    st = ctx.stats()
    ctx.close()
    for k, (a, b) in enumerate(got):
        assert_bitwise(a[:, :3], ref[0][:, :3], f"frame {k} rgba")
        assert np.array_equal(b, ref[1]), f"frame {k} g_data"
    assert st["svc_jobs"] == len(jobs) and st["svc_sessions"] >= 1 and st["svc_running"] == 0
    assert st["samples"] == len(jobs) * W * H * 16
    assert st["launches"] == len(jobs)


@pytest.mark.parametrize("full", [0, 1])
@pytest.mark.parametrize("mode", [0, 1])
def test_service_lds_tree_sessions_equal_launched_frames(spt, monkeypatch, mode, full):
    """A 10 000-sphere stress scene (config 5's generator; its 2 026-node tree takes the
    LDS lane walk) through the service (SPT_SVC_LDS=1, opt-in): the session runs
    render_kernel_svc_lds (1 024-
    thread blocks, the node table in LDS, the resumable lane walk; at most 2 blocks per CU)
    and every frame and rank share equals its launched render bit for bit -- the launched
    LDS kernel is pinned against brute force and the oracle by test_gpu_parity.py."""
    import torch
    monkeypatch.setenv("SPT_SVC_FULL_GRID", str(full))
    monkeypatch.setenv("SPT_SVC_LDS", "1")
    W, H = 320, 180
    ctx = spt.Context(0)
    ctx.set_scene(spt.generate_stress(5, 10000))
    ctx.set_camera(spt.camera_basis(EYE, LOOK, UP), EYE, SKY)
    ctx.set_params(W, H, 8, 50, 11)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = [(0, H, 1, 1, 0, 0, W)] * 3 + [(0, H, 4, 3, p, 0, W) for p in range(3)] + [(5, 61, 1, 1, 0, 17, 250)]
    ref = render_frames(ctx, jobs, W, H, mode, streams, service=False)
    ctx.reset_stats()
    got = render_frames(ctx, jobs, W, H, mode, streams, service=True)
    st = ctx.stats()
    ctx.close()
    for k, ((a, b), (ra, rb)) in enumerate(zip(got, ref)):
        assert_bitwise(a[:, :3], ra[:, :3], f"job {k} {jobs[k]} rgba")
        assert np.array_equal(b, rb), f"job {k} {jobs[k]} g_data"
    assert st["svc_jobs"] == len(jobs) and st["svc_sessions"] >= 1 and st["svc_running"] == 0
    assert st["svc_watchdog_exits"] == 0
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    # the LDS-tree session's grid: 1 024-thread blocks, one per CU (two with the full grid)
    assert st["svc_grid_blocks"] == (2 if full else 1) * n_cu


def test_service_rank_shares_and_regions(spt, golden_scenes):
    """Interleaved strips (the bench's rank shares), odd rectangles and tiny regions, many
    jobs in flight at once (more than 64 of them: the job search's second step)."""
    import torch
    W, H = 240, 160
    ctx = make_ctx(spt, golden_scenes, W, H, 8, 50, seed=7)
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = [(0, H, 4, 8, p, 0, W) for p in range(8)] + [(0, H, 8, 3, p, 17, 201) for p in range(3)]
    jobs += [(y, y + 3, 1, 1, 0, x, x + 5) for y in range(0, 150, 13) for x in range(0, 230, 37)]
    jobs += [(11, 12, 1, 1, 0, 23, 24)] * 3
    assert len(jobs) > 64
    ref = render_frames(ctx, jobs, W, H, 0, streams, service=False)
    got = render_frames(ctx, jobs, W, H, 0, streams, service=True)
    st = ctx.stats()
    ctx.close()
    for k, ((a, b), (ra, rb)) in enumerate(zip(got, ref)):
        assert_bitwise(a[:, :3], ra[:, :3], f"job {k} {jobs[k]} rgba")
        bad = np.nonzero(b != rb)[0]
        assert not len(bad), (f"job {k} {jobs[k]} g_data: {len(bad)} bytes differ, rows "
                              f"{sorted(set((H - 1 - bad // (3 * W)).tolist()))[:12]}, got {b[bad[:8]]} want {rb[bad[:8]]}")
    assert st["svc_watchdog_exits"] == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_service_sample_batches_fold_in_order(spt, golden_scenes, mode):
    """A workspace smaller than the frame's sample words: each frame is several jobs (one
    per sample batch), folded in order into the accumulator."""
    import torch
    W, H = 200, 120
    ctx = make_ctx(spt, golden_scenes, W, H, 24, 50, seed=2)
    streams = [torch.cuda.Stream()]
    jobs = [(0, H, 1, 1, 0, 0, W)] * 2
    ref = render_frames(ctx, jobs[:1], W, H, mode, streams, service=False)[0]
    ctx.set_workspace(W * H * 5 * 4 * (2 if mode else 1))  # 5 samples per batch: 5 batches
    got = render_frames(ctx, jobs, W, H, mode, streams, service=True)
    st = ctx.stats()
    ctx.close()
    for k, (a, b) in enumerate(got):
        assert_bitwise(a[:, :3], ref[0][:, :3], f"frame {k}")
        assert np.array_equal(b, ref[1])
    assert st["svc_jobs"] >= 2 * 5


def test_service_restarts_after_a_pause_and_a_setter(spt, golden_scenes):
    """A pause longer than the session's idle limit (its waves leave; the host starts a
    new session), a camera change between frames (the session ends), then more frames."""
    import torch
    W, H = 160, 96
    ctx = make_ctx(spt, golden_scenes, W, H, 8, 50, seed=4)
    st0 = torch.cuda.Stream()
    job = [(0, H, 1, 1, 0, 0, W)]
    ref = render_frames(ctx, job, W, H, 0, [st0], service=False)[0]
    ctx.service_start()
    outs = []
    for k in range(3):
        rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()  # the fill (current stream) before the render stream writes
        ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), 0, st0.cuda_stream)
        st0.synchronize()  # the stream only: the session stays resident
        outs.append(rgba.cpu().numpy())
        time.sleep(0.7)  # > kSvcIdleTicks (0.5 s): the session's waves leave
    view2 = spt.camera_basis([0.5, 1.2, -3, 0], LOOK, UP)
    ctx.set_camera(view2, EYE, SKY)
    rgba2 = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba2.data_ptr(), 0, st0.cuda_stream)
    ctx.service_stop()
    st = ctx.stats()
    ctx.synchronize()
    torch.cuda.synchronize()
    got2 = rgba2.cpu().numpy()
    ctx.set_camera(view2, EYE, SKY)
    want2 = render_frames(ctx, job, W, H, 0, [st0], service=False)[0]
    ctx.close()
    for k, a in enumerate(outs):
        assert_bitwise(a[:, :3], ref[0][:, :3], f"frame {k} after a pause")
    assert_bitwise(got2[:, :3], want2[0][:, :3], "frame after set_camera")
    assert st["svc_sessions"] >= 4 and st["svc_watchdog_exits"] >= 2


def test_service_host_slot_calls(spt, golden_scenes, monkeypatch):
    """Unbatched host calls (SPT_BATCH=0: one host slot and stream per call, from several
    threads) go through the service too."""
    import threading
    monkeypatch.setenv("SPT_BATCH", "0")
    W, H = 200, 120
    ctx = make_ctx(spt, golden_scenes, W, H, 6, 50, seed=9)
    tiles = [(y, y + 40, x, x + 50) for y in range(0, H, 40) for x in range(0, W, 50)]
    want = np.zeros(W * H * 3, np.uint8)
    for t in tiles:
        ctx.render_segment(*t, want)
    ctx.service_start()
    got = np.zeros(W * H * 3, np.uint8)
    th = [threading.Thread(target=ctx.render_segment, args=(*t, got)) for t in tiles]
    for t in th:
        t.start()
    for t in th:
        t.join()
    st = ctx.stats()
    ctx.service_stop()
    ctx.close()
    assert np.array_equal(got, want)
    assert st["svc_jobs"] == len(tiles)


def _hooks():
    """The test-only kernels (tests/cpp/spt_testhooks.hip, built by the csrc Makefile)."""
    import ctypes
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simplepathtracer_amd", "lib",
                        "libspt_testhooks.so")
    h = ctypes.CDLL(path)
    h.spt_test_blocker.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    h.spt_test_blocker.restype = ctypes.c_int
    h.spt_test_blocker_vgprs.argtypes = [ctypes.c_void_p]
    h.spt_test_blocker_vgprs.restype = ctypes.c_int
    return h


@pytest.mark.parametrize("full", [0, 1])
@pytest.mark.parametrize("mode", [0, 1])
def test_service_ring_wrap_behind_blockers(spt, golden_scenes, monkeypatch, mode, full):
    """Liveness.  A 64 MiB slot ring wraps every few
    jobs, and on each caller stream, ahead of every render's fold, sits a kernel that cannot
    be resident beside a session (512 threads x 256 VGPRs, standing in for RCCL's gather
    kernels): so a fold cannot run while the session does.  A publication
    whose ring words such a fold still reads must not be held inside the running session
    (the fold waits for the blocker, the blocker for the session to end, the session for
    the publication: round 4's build hung here); the host ends the session and the next
    session's launch waits for the fold instead.  Every frame bit-identical to a launch."""
    import ctypes
    import os

    import torch
    monkeypatch.setenv("SPT_SVC_RING_MB", "64")
    monkeypatch.setenv("SPT_SVC_TIMEOUT_MS", "30000")
    monkeypatch.setenv("SPT_SVC_FULL_GRID", str(full))  # 1: no fold can run inside a session at all
    hooks = _hooks()
    vg = ctypes.c_int(0)
    assert hooks.spt_test_blocker_vgprs(ctypes.byref(vg)) == 0 and vg.value == 256
    W, H, spp = 320, 200, 16  # 1.02 M sample words (4.1 MB segment, 8.2 MB task): 15 / 7 jobs per ring
    ctx = make_ctx(spt, golden_scenes, W, H, spp, 50, seed=5)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ref = render_frames(ctx, [(0, H, 1, 1, 0, 0, W)], W, H, mode, streams, service=False)[0]
    n = 36
    outs = [torch.zeros((W * H, 4), dtype=torch.float32, device="cuda") for _ in range(n)]
    g8s = [torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda") for _ in range(n)]
    ran = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.reset_stats()
    ctx.service_start()
    block_us = int(os.environ.get("SPT_TEST_BLOCK_US", "2000"))  # 0: no blockers (diagnostics)
    for k in range(n):
        s = streams[k % 2]
        if block_us:
            assert hooks.spt_test_blocker(ctypes.c_void_p(s.cuda_stream), block_us, 8, ctypes.c_void_p(ran.data_ptr())) == 0
        ctx.render_rows_async(mode, 0, H, 1, 1, 0, 0, W, outs[k].data_ptr(), g8s[k].data_ptr(), s.cuda_stream)
    ctx.service_stop()
    st = ctx.stats()
    ctx.synchronize()
    torch.cuda.synchronize()
    ctx.close()
    for k in range(n):
        assert_bitwise(outs[k].cpu().numpy()[:, :3], ref[0][:, :3], f"frame {k}")
        assert np.array_equal(g8s[k].cpu().numpy(), ref[1]), f"frame {k} g_data"
    assert int(ran.item()) == (8 * n if block_us else 0)
    assert st["svc_jobs"] == n and st["svc_running"] == 0
    # the ring wrapped onto words whose folds were still held by the blockers
    assert st["svc_flow_restarts"] >= 1 and st["svc_sessions"] >= 2, st


def test_service_publish_delayed_past_the_idle_limit(spt, golden_scenes, monkeypatch):
    """Liveness: every publication is held 0.7 s between its commit and its publication
    (fault injection, SPT_SVC_TEST_PUB_DELAY_US), longer than a wave may idle
    (kSvcIdleTicks, 0.5 s).  The waves may not leave while the host has committed jobs the
    device has not published (the closing handshake, spt_internal.h): every frame is
    rendered, bit-identical, and no session ends through its watchdog -- the second
    publication finds the closing flag the idle waves raised and goes to a fresh session,
    the first one ending on its stop flag.  (Round 4's waves left at 0.5 s and the fold of
    a frame published later waited forever.)"""
    import torch
    monkeypatch.setenv("SPT_SVC_TEST_PUB_DELAY_US", "700000")
    monkeypatch.setenv("SPT_SVC_TIMEOUT_MS", "30000")
    W, H = 160, 96
    ctx = make_ctx(spt, golden_scenes, W, H, 8, 50, seed=6)
    st0 = torch.cuda.Stream()
    job = [(0, H, 1, 1, 0, 0, W)]
    ref = render_frames(ctx, job, W, H, 0, [st0], service=False)[0]
    ctx.reset_stats()
    t0 = time.perf_counter()
    got = render_frames(ctx, job * 2, W, H, 0, [st0], service=True)
    dt = time.perf_counter() - t0
    st = ctx.stats()
    ctx.close()
    for k, (a, b) in enumerate(got):
        assert_bitwise(a[:, :3], ref[0][:, :3], f"frame {k}")
        assert np.array_equal(b, ref[1])
    assert dt > 1.3  # both publications were really held
    assert st["svc_jobs"] == 2 and st["svc_watchdog_exits"] == 0, st
    assert st["svc_sessions"] == 1 + st["svc_closing_restarts"] and st["svc_closing_restarts"] <= 1, st
