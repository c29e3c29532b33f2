"""Paths added in rounds 4 and 5, checked against the oracle directly and not only
against the launched path: regions rendered as jobs of the resident
render service, the drop-in's tiling read-ahead (spt_batch.cpp SpecFrame,
DESIGN.md §5) and launches on CU-masked streams (spt_set_reserved_cus), each compared bit
for bit with the CPU restatement (oracle/: RenderSegment / RenderSegmentTask,
SingleThreadPathTracer.hpp:118-136 / TaskBasedPathTracer.hpp:61-210, and
RenderImageParallelMain's tiling, Renderer.hpp:257-302) on the same seeded inputs, float
pixels and g_data bytes."""
import threading

import numpy as np
import pytest

from test_gpu_parity import EYE, SKY, assert_bitwise, oscene_from, scene_from, setup

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


@pytest.mark.parametrize("task", [False, True])
def test_service_jobs_vs_oracle(spt, oracle, golden_scenes, task):
    """Three regions of the random scene (a window, a ragged strip, a single row) rendered
    by host calls from three threads while one service session is resident."""
    W, H, spp = 320, 200, 8
    regions = [(40, 72, 100, 164), (121, 134, 3, 317), (199, 200, 0, 320)]
    ctx = spt.Context(0)
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, spp, 50, seed=7, view=golden_scenes["view"])
    g = np.full(W * H * 3, 0x5A, np.uint8)
    got = [None] * len(regions)
    ctx.service_start()

    def job(k):
        got[k] = ctx.render_segment(*regions[k], g_data=g, task=task)

    th = [threading.Thread(target=job, args=(k,)) for k in range(len(regions))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ctx.service_stop()
    st = ctx.stats()
    ctx.close()
    assert st["svc_jobs"] == len(regions) and st["svc_running"] == 0, st
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, spp, 50, 7)
    gw = np.full(W * H * 3, 0x5A, np.uint8)
    for k, (yB, yE, xB, xE) in enumerate(regions):
        want, _ = oracle.render_segment(sc, fr, yB, yE, xB, xE, task=task, rgb8=gw)
        assert_bitwise(got[k][:, :3], want[:, :3], f"service region {k}")
    assert np.array_equal(g, gw), f"g_data: {np.count_nonzero(g != gw)} bytes differ"


@pytest.mark.parametrize("task", [False, True])
def test_readahead_tiling_vs_oracle(spt, oracle, golden_scenes, task):
    """The reference's tc = 4 tiling of a 240 x 160 frame, g_data only, four calls at once:
    the first frame arms the tiling, the next two are served from the read-ahead; every
    frame's bytes equal the oracle's RenderImageParallelMain."""
    W, H, spp, tc = 240, 160, 6, 4
    ctx = spt.Context(0)
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, spp, 50, seed=3, view=golden_scenes["view"])
    sw, sh = W // tc, H // tc
    tiles = [(sh * j, sh * j + sh, sw * i, sw * i + sw) for j in range(tc) for i in range(tc)]

    def frame():
        g = np.zeros(W * H * 3, np.uint8)
        sem = threading.Semaphore(tc)
        th = []

        def job(t):
            try:
                ctx.render_segment(*t, g_data=g, task=task, rgba=False)
            finally:
                sem.release()

        for t in tiles:
            sem.acquire()
            th.append(threading.Thread(target=job, args=(t,)))
            th[-1].start()
        for t in th:
            t.join()
        return g

    frames = [frame()]
    ctx.reset_stats()
    frames += [frame(), frame()]
    st = ctx.stats()
    ctx.close()
    assert st["batches"] == 2 * 4 and st["batched_calls"] == 2 * tc * tc, st  # served by the read-ahead
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, spp, 50, 3)
    _, want8 = oracle.render_image_parallel(sc, fr, tc, mode=1 if task else 0, want_rgba=False)
    for k, g in enumerate(frames):
        assert np.array_equal(g, want8), f"frame {k}: {np.count_nonzero(g != want8)} bytes differ"


def test_reserved_cus_region_vs_oracle(spt, oracle, golden_scenes):
    """A launched render on the CU-masked stream (spt_set_reserved_cus, 32 CUs kept free)."""
    W, H, spp = 320, 200, 8
    ctx = spt.Context(0)
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, spp, 50, seed=11, view=golden_scenes["view"])
    ctx.set_reserved_cus(32)
    g = np.zeros(W * H * 3, np.uint8)
    got = ctx.render_segment(20, 180, 30, 290, g_data=g)
    ctx.close()
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, spp, 50, 11)
    gw = np.zeros(W * H * 3, np.uint8)
    want, _ = oracle.render_segment(sc, fr, 20, 180, 30, 290, rgb8=gw)
    assert_bitwise(got[:, :3], want[:, :3], "reserved-CU region")
    assert np.array_equal(g, gw)


@pytest.mark.parametrize("w,h,spp,bounces", [(1, 1, 1, 1), (7, 3, 3, 2), (9, 17, 1, 50), (65, 1, 2, 5), (1, 70, 4, 3)])
@pytest.mark.parametrize("task", [False, True])
@pytest.mark.parametrize("engine", ["megakernel", "wavefront"])
def test_tiny_and_thin_frames_vs_oracle(spt, oracle, golden_scenes, w, h, spp, bounces, task, engine):
    """Whole frames smaller than one 8x8 tile, one pixel wide or high, a single sample, a
    single bounce: the tile decomposition's ragged edges (ts_item / ts_slot_base) and the
    primary batches' partial blocks against RenderSegment / RenderSegmentTask, on both
    engines (the megakernel and the wavefront queue workers)."""
    ctx = spt.Context(0)
    if engine == "wavefront":
        ctx.set_engine(spt._native.ENGINE_WAVEFRONT)
    setup(ctx, scene_from(spt, golden_scenes, "random"), w, h, spp, bounces, seed=13, view=golden_scenes["view"])
    g = np.zeros(w * h * 3, np.uint8)
    got = ctx.render_segment(0, h, 0, w, g_data=g, task=task)
    ctx.close()
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, w, h, spp, bounces, 13)
    gw = np.zeros(w * h * 3, np.uint8)
    want, _ = oracle.render_segment(sc, fr, 0, h, 0, w, task=task, rgb8=gw)
    assert_bitwise(got[:, :3], want[:, :3], f"{w}x{h}")
    assert np.array_equal(g, gw)
