"""GPU tests of the drop-in's tiling read-ahead (spt_batch.cpp SpecFrame):
RenderSegment / RenderSegmentTask calls over the reference's tc x tc tiling
(Renderer.hpp:264-273, MakeRenderSegmentData), g_data only, are served from one
read-ahead render of the whole tiling, once the caller has called every tile of that
tiling (the tiling is armed).  Every output byte must equal a plain render, a lone
first-tile call must write only its own rows and start no read-ahead, a frame whose
first call is another tile (the reference's detached threads keep no order) must be
served too, and a setter between frames must not serve a stale frame.  The drop-in's
setting (spt_prepare_dropin) arms a tiling at its first call instead, so that the first
frame is served too."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EYE, LOOK, UP, SKY = [0, 1, -3, 0], [0, 1, 0, 0], [0, 1, 0, 0], [137, 207, 240, 0]


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


def make_ctx(spt, golden_scenes, w, h, spp, seed=1):
    gs = golden_scenes
    c = spt.Context(0)
    c.set_scene(spt.Scene(*(gs[f"random_{k}"] for k in ("centers", "radii", "colors", "materials", "fuzz"))))
    c.set_camera(spt.camera_basis(EYE, LOOK, UP), EYE, SKY)
    c.set_params(w, h, spp, 50, seed)
    return c


def tiles(W, H, tc):
    sw, sh = W // tc, H // tc
    return [(sh * j, sh * j + sh, sw * i, sw * i + sw) for j in range(tc) for i in range(tc)]


def render_tiling(ctx, W, H, tc, task, threads):
    """RenderImageParallelMain's pattern: every tile, at most `threads` calls at once."""
    g = np.zeros(W * H * 3, np.uint8)
    sem = threading.Semaphore(threads)
    err = []

    def job(t):
        try:
            ctx.render_segment(*t, g_data=g, task=task, rgba=False)
        except Exception as e:  # noqa: BLE001
            err.append(e)
        finally:
            sem.release()

    th = []
    for t in tiles(W, H, tc):
        sem.acquire()
        th.append(threading.Thread(target=job, args=(t,)))
        th[-1].start()
    for t in th:
        t.join()
    assert not err, err
    return g


@pytest.mark.parametrize("task", [False, True])
def test_tiling_served_from_readahead_equals_plain_calls(spt, golden_scenes, monkeypatch, task):
    W, H, spp, tc = 240, 160, 6, 4
    ctx = make_ctx(spt, golden_scenes, W, H, spp, seed=5)
    frames = [render_tiling(ctx, W, H, tc, task, 4)]  # plain calls: arms the tiling
    ctx.reset_stats()
    frames += [render_tiling(ctx, W, H, tc, task, 4) for _ in range(2)]
    st = ctx.stats()
    ctx.close()
    monkeypatch.setenv("SPT_READAHEAD", "0")
    plain = make_ctx(spt, golden_scenes, W, H, spp, seed=5)
    want = np.zeros(W * H * 3, np.uint8)
    for t in tiles(W, H, tc):
        plain.render_segment(*t, g_data=want, task=task, rgba=False)
    plain.close()
    for k, g in enumerate(frames):
        assert np.array_equal(g, want), f"frame {k}: {np.count_nonzero(g != want)} bytes differ"
    # min(4, tc) read-ahead launches per frame (SPT_READAHEAD_PARTS), every tile in them
    assert st["batches"] == 2 * min(4, tc) and st["batched_calls"] == 2 * tc * tc


def test_lone_first_tile_writes_only_its_rows(spt, golden_scenes):
    W, H, spp = 200, 120, 4
    ctx = make_ctx(spt, golden_scenes, W, H, spp)
    g = np.zeros(W * H * 3, np.uint8)
    for _ in range(2):  # tile (0, 0) of tc = 2, twice: the tiling never arms
        ctx.render_segment(0, H // 2, 0, W // 2, g_data=g, rgba=False)
    st = ctx.stats()
    assert st["batched_calls"] == 2 and st["samples"] == 2 * (W // 2) * (H // 2) * spp  # no read-ahead
    want = np.zeros(W * H * 3, np.uint8)
    ref = make_ctx(spt, golden_scenes, W, H, spp)
    ref.render_segment(0, H // 2, 0, W // 2, g_data=want)  # rgba requested: no read-ahead
    ref.close()
    ctx.close()
    assert np.array_equal(g, want)
    img = g.reshape(H, W, 3)
    assert not img[: H // 2].any() and not img[H // 2:, W // 2:].any()  # g_data row r = image row H-1-r


def test_setter_between_frames_is_not_served_stale(spt, golden_scenes):
    W, H, spp, tc = 160, 96, 4, 2
    ctx = make_ctx(spt, golden_scenes, W, H, spp)
    render_tiling(ctx, W, H, tc, False, 2)
    # start a frame, then change the camera before its other tiles are asked for
    g = np.zeros(W * H * 3, np.uint8)
    ctx.render_segment(*tiles(W, H, tc)[0], g_data=g, rgba=False)
    ctx.set_camera(spt.camera_basis([0.5, 1.2, -3, 0], LOOK, UP), EYE, SKY)
    for t in tiles(W, H, tc)[1:]:
        ctx.render_segment(*t, g_data=g, rgba=False)
    ctx.close()
    ref = make_ctx(spt, golden_scenes, W, H, spp)
    ref.set_camera(spt.camera_basis([0.5, 1.2, -3, 0], LOOK, UP), EYE, SKY)
    want2 = np.zeros(W * H * 3, np.uint8)
    for t in tiles(W, H, tc)[1:]:
        ref.render_segment(*t, g_data=want2)
    ref.close()
    img, ref_img = g.reshape(H, W, 3), want2.reshape(H, W, 3)
    # tiles 1.. (the new camera) match a plain render with the new camera
    assert np.array_equal(img[: H // 2], ref_img[: H // 2]) and np.array_equal(img[H // 2:, W // 2:], ref_img[H // 2:, W // 2:])


@pytest.mark.parametrize("first", [(0, 1), (1, 1), (3, 2)])
def test_readahead_starts_at_any_tile(spt, golden_scenes, first):
    """Renderer.hpp:282-290 detaches its RenderJob threads, so a frame's first call may be
    any tile: once armed, the first call of a frame -- tile (i, j) = `first` here -- starts
    the read-ahead, every tile of the frame is served from it (one frame's launches, no
    plain render), and the bytes equal plain calls."""
    W, H, spp, tc = 240, 160, 4, 4
    ctx = make_ctx(spt, golden_scenes, W, H, spp, seed=8)
    want = render_tiling(ctx, W, H, tc, False, 4)  # plain calls: arms the tiling
    ctx.reset_stats()
    order = tiles(W, H, tc)
    sw, sh = W // tc, H // tc
    i, j = first
    lead = (sh * j, sh * j + sh, sw * i, sw * i + sw)
    order.remove(lead)
    g = np.zeros(W * H * 3, np.uint8)
    ctx.render_segment(*lead, g_data=g, rgba=False)
    for t in reversed(order):
        ctx.render_segment(*t, g_data=g, rgba=False)
    st = ctx.stats()
    ctx.close()
    assert np.array_equal(g, want), f"{np.count_nonzero(g != want)} bytes differ"
    assert st["batches"] == min(4, tc) and st["batched_calls"] == tc * tc and st["samples"] == W * H * spp


@pytest.mark.parametrize("task", [False, True])
def test_dropin_first_frame_served_from_readahead(spt, golden_scenes, monkeypatch, task):
    """The drop-in (spt_prepare_dropin, which the C++ shim calls) arms the read-ahead at a
    tiling's first call (RenderImageParallelMain's detached threads arrive in no fixed
    order), so MainLoop's one frame per
    process (Renderer.hpp:335-344) is rendered whole in the read-ahead's launches.  Its bytes
    equal plain calls, whichever tile comes first; a lone tile (0, 0) still writes only its
    own rows (the rest of the frame is rendered but not copied); SPT_READAHEAD_FIRST=0 keeps
    the first frame tile by tile."""
    W, H, spp, tc = 240, 160, 4, 4
    monkeypatch.setenv("SPT_READAHEAD", "0")
    plain = make_ctx(spt, golden_scenes, W, H, spp, seed=6)
    want = np.zeros(W * H * 3, np.uint8)
    for t in tiles(W, H, tc):
        plain.render_segment(*t, g_data=want, task=task, rgba=False)
    plain.close()
    monkeypatch.delenv("SPT_READAHEAD")
    ctx = make_ctx(spt, golden_scenes, W, H, spp, seed=6)
    ctx.prepare_dropin()
    ctx.reset_stats()
    g = render_tiling(ctx, W, H, tc, task, 4)
    st = ctx.stats()
    ctx.close()
    assert np.array_equal(g, want), f"{np.count_nonzero(g != want)} bytes differ"
    assert st["batches"] == min(4, tc) and st["batched_calls"] == tc * tc and st["samples"] == W * H * spp
    # a lone tile (0, 0): only its rows reach g_data
    lone = make_ctx(spt, golden_scenes, W, H, spp, seed=6)
    lone.prepare_dropin()
    g1 = np.zeros(W * H * 3, np.uint8)
    lone.render_segment(*tiles(W, H, tc)[0], g_data=g1, task=task, rgba=False)
    lone.close()
    img, ref = g1.reshape(H, W, 3), want.reshape(H, W, 3)
    sw, sh = W // tc, H // tc
    # tile (0, 0) = image rows [0, sh), columns [0, sw) = g_data rows H-sh.. H-1
    assert np.array_equal(img[H - sh:, :sw], ref[H - sh:, :sw])
    img2 = img.copy()
    img2[H - sh:, :sw] = 0
    assert not img2.any()
    monkeypatch.setenv("SPT_READAHEAD_FIRST", "0")
    off = make_ctx(spt, golden_scenes, W, H, spp, seed=6)
    off.prepare_dropin()
    off.reset_stats()
    g2 = render_tiling(off, W, H, tc, task, 4)
    st2 = off.stats()
    off.close()
    assert np.array_equal(g2, want)
    assert st2["samples"] == W * H * spp and st2["batched_calls"] == tc * tc and st2["batches"] >= 1


def test_late_call_is_served_without_another_frame(spt, golden_scenes):
    """A RenderJob thread that starts after its frame's final wait (Renderer.hpp:242-255,
    282-292) calls its tile after the next frame has begun: that frame's read-ahead serves
    it, and the next frame's own call of the same tile is served as an owed tile -- two
    read-ahead frames for the two frames, not three -- with the bytes of plain calls."""
    W, H, spp, tc = 160, 96, 4, 2
    ctx = make_ctx(spt, golden_scenes, W, H, spp, seed=9)
    want = render_tiling(ctx, W, H, tc, False, 2)  # plain calls: arms the tiling
    ctx.reset_stats()
    a, b, c, d = tiles(W, H, tc)
    g1 = np.zeros(W * H * 3, np.uint8)
    g2 = np.zeros(W * H * 3, np.uint8)
    for t in (a, b, c):  # frame 1 without its late tile d
        ctx.render_segment(*t, g_data=g1, rgba=False)
    ctx.render_segment(*a, g_data=g2, rgba=False)  # frame 2 begins
    ctx.render_segment(*d, g_data=g1, rgba=False)  # frame 1's late call
    for t in (b, c, d):
        ctx.render_segment(*t, g_data=g2, rgba=False)
    st = ctx.stats()
    ctx.close()
    assert np.array_equal(g1, want) and np.array_equal(g2, want)
    parts = min(4, tc)
    assert st["batches"] == 2 * parts and st["batched_calls"] == 2 * tc * tc, st
