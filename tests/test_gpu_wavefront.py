"""GPU parity tests of the wavefront engine (spt_wavefront.hip):
RenderSegmentTask's material-queue design as block queue workers (cast, sort by
material in LDS, shade, compact per pass).  It shares the megakernel's per-path
code, so frames, ray counts and task-mode drops must be bit-identical to the
goldens, the oracle and the megakernel."""
import os

import numpy as np
import pytest

from test_gpu_parity import EYE, LOOK, SKY, UP, _mirror_lattice, assert_bitwise, scene_from, setup

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


@pytest.fixture(scope="module")
def wctx(spt):
    c = spt.Context(0)
    c.set_engine(spt._native.ENGINE_WAVEFRONT)
    yield c
    c.close()


@pytest.fixture(scope="module")
def mctx(spt):
    c = spt.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", ["cornell3", "reference"])
@pytest.mark.parametrize("task", [False, True])
def test_config1_frames_match_golden(spt, wctx, golden, golden_scenes, name, task):
    setup(wctx, scene_from(spt, golden_scenes, name), 200, 100, 4, 8)
    g = np.zeros(200 * 100 * 3, np.uint8)
    if not task:
        rgba = wctx.render_segment(0, 100, 0, 200, g)
        assert_bitwise(rgba[:, :3], golden[f"c1_{name}_rgba"][:, :3], f"C1 {name}")
        assert np.array_equal(g, golden[f"c1_{name}_rgb8"])
        return
    out = np.zeros((100, 200, 4), np.float32)
    for ty in range(0, 100, 50):
        for tx in range(0, 200, 50):
            out[ty:ty + 50, tx:tx + 50] = wctx.render_segment(ty, ty + 50, tx, tx + 50, g, task=True).reshape(50, 50, 4)
    assert_bitwise(out.reshape(-1, 4)[:, :3], golden[f"c1_{name}_task_rgba"][:, :3], f"C1 {name} task")
    assert np.array_equal(g, golden[f"c1_{name}_task_rgb8"])


def test_config2_window_matches_golden(spt, wctx, golden, golden_scenes):
    setup(wctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 100, 50)
    win = wctx.render_segment(400, 416, 592, 608)
    assert_bitwise(win[:, :3], golden["c2_window_400_592_rgba"][:, :3], "C2 window")


@pytest.mark.parametrize("scene_name", ["random", "stress"])
def test_full_frame_equals_megakernel(spt, wctx, mctx, golden_scenes, scene_name):
    """Same frame, same ray count from both engines (flat cluster list and tree)."""
    if scene_name == "random":
        scene, W, H, spp = scene_from(spt, golden_scenes, "random"), 1200, 800, 8
    else:
        scene, W, H, spp = spt.generate_stress(3, 3000), 480, 270, 4
    out = {}
    for c in (wctx, mctx):
        setup(c, scene, W, H, spp, 50)
        c.reset_stats()
        g = np.zeros(W * H * 3, np.uint8)
        out[id(c)] = (c.render_segment(0, H, 0, W, g), g, c.stats())
    (wf, wg, ws), (mk, mg, ms) = out[id(wctx)], out[id(mctx)]
    assert_bitwise(wf, mk, f"{scene_name}: wavefront vs megakernel")
    assert np.array_equal(wg, mg)
    assert ws["casts"] == ms["casts"] and ws["samples"] == ms["samples"] == W * H * spp


def test_task_mode_drops_match_megakernel(spt, wctx, mctx, oracle):
    arrays = _mirror_lattice()
    res = []
    for c in (wctx, mctx):
        setup(c, spt.Scene(*arrays), 64, 64, 16, 8, seed=9)
        c.reset_stats()
        res.append((c.render_segment(0, 64, 0, 64, task=True), c.stats()["dropped"]))
    assert res[0][1] == res[1][1] > 0
    assert_bitwise(res[0][0], res[1][0], "task mode with drops")
    osc = oracle.OracleScene(*arrays)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 64, 64, 16, 8, 9)
    want, _ = oracle.render_segment(osc, fr, 0, 64, 0, 64, task=True)
    assert_bitwise(res[0][0][:, :3], want[:, :3], "task mode vs oracle")


@pytest.mark.parametrize("queue", [256, 2048])
def test_small_queue_and_sample_batches(spt, mctx, golden_scenes, queue):
    """Two block queues of 256 or one of 2048 rays (many top-ups and passes) and a
    workspace forcing sample batches still give the megakernel's frame."""
    old = {k: os.environ.get(k) for k in ("SPT_WF_CAP", "SPT_WF_QUEUE")}
    os.environ["SPT_WF_CAP"] = "2048" if queue == 2048 else "512"
    os.environ["SPT_WF_QUEUE"] = str(queue)
    try:
        c = spt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        c.set_engine(spt._native.ENGINE_WAVEFRONT)
        scene = scene_from(spt, golden_scenes, "random")
        setup(c, scene, 96, 64, 12, 50)
        c.set_workspace(96 * 64 * 5 * 4)  # 5 samples per batch (4-byte slots)
        got = c.render_segment(0, 64, 0, 96)
        setup(mctx, scene, 96, 64, 12, 50)
        assert_bitwise(got, mctx.render_segment(0, 64, 0, 96), "small queue + batches")
    finally:
        c.close()


def test_device_launch_returns_before_the_frame(spt, wctx, mctx, golden_scenes):
    """No host round trip inside a render: a device-resident config-2 launch returns
    while its stream is still busy (queue lengths never leave the GPU), and the frame
    equals the megakernel's."""
    import torch
    W, H = 1200, 800
    scene = scene_from(spt, golden_scenes, "random")
    outs = []
    for c in (wctx, mctx):
        setup(c, scene, W, H, 32, 50)
        rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        st = torch.cuda.Stream()
        torch.cuda.synchronize()  # the fill (current stream) before the render stream writes
        c.render_rows_async(spt.MODE_SEGMENT, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), 0, st.cuda_stream)
        busy = not st.query()
        st.synchronize()
        outs.append((rgba.cpu().numpy(), busy))
    assert outs[0][1], "the wavefront render call waited for its own launch"
    assert_bitwise(outs[0][0], outs[1][0], "device launch: wavefront vs megakernel")


def test_engine_argument_is_checked(spt, wctx):
    with pytest.raises(spt.SptError):
        wctx.set_engine(7)
