"""GPU tests of reserved CUs (spt_set_reserved_cus, DESIGN.md §5 "Reserved CUs"): launched
renders on the context's CU-masked streams must give frames bit-identical to unmasked
ones (the launch only shrinks its persistent grid; the per-sample work and the fold
order are unchanged), and a collective-sized kernel (tests/cpp/spt_testhooks.hip's
blocker: 512-thread blocks of 256-VGPR waves, like RCCL's for gfx950) queued on another
stream while a long render runs must start on the reserved CUs and finish long before
the render does."""
import ctypes

import numpy as np
import pytest

from test_gpu_service import _hooks, assert_bitwise, render_frames

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


def config2_ctx(spt, W, H, spp, bounces=50):
    c = spt.Context(0)
    c.set_scene(spt.generate_spheres(1))
    c.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
    c.set_params(W, H, spp, bounces, 1)
    return c


@pytest.mark.parametrize("mode", [0, 1])
def test_reserved_frames_identical(spt, mode):
    import torch
    W, H, spp = 320, 200, 16
    jobs = [(0, H, 1, 1, 0, 0, W),            # whole frame
            (0, H, 4, 2, 1, 0, W),            # a rank's share of 4-row strips
            (37, 151, 1, 1, 0, 13, 301)]      # a ragged region
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ctx = config2_ctx(spt, W, H, spp)
    ref = render_frames(ctx, jobs, W, H, mode, streams, service=False)
    for n in (8, 64, 255):
        ctx.set_reserved_cus(n)
        got = render_frames(ctx, jobs, W, H, mode, streams, service=False)
        for k, ((a, b), (ra, rb)) in enumerate(zip(got, ref)):
            assert_bitwise(a[:, :3], ra[:, :3], f"reserve {n}, job {k}")
            assert np.array_equal(b, rb), f"reserve {n}, job {k} g_data"
    ctx.set_reserved_cus(0)
    got = render_frames(ctx, jobs[:1], W, H, mode, streams, service=False)
    assert_bitwise(got[0][0][:, :3], ref[0][0][:, :3], "reserve back to 0")
    ctx.close()


def test_reserved_count_checked(spt):
    ctx = config2_ctx(spt, 64, 64, 1)
    with pytest.raises(Exception):
        ctx.set_reserved_cus(1 << 20)
    ctx.set_reserved_cus(0)
    ctx.close()


def test_collective_sized_kernel_runs_beside_render(spt):
    """A ~20 ms render on stream A with 32 reserved CUs (one per shader engine of each
    XCC: the mask's last bits, tools/cu_mask_probe.py); 8 blocker blocks of 1 ms queued on
    stream B just after it must end within the render's first half.  Without the
    reservation they wait for the render to end (printed for comparison); with one CU per
    XCC (8) some still do -- a block waits for room in the shader engine it is sent to."""
    import torch
    W, H, spp = 1200, 800, 400
    hooks = _hooks()
    ctx = config2_ctx(spt, W, H, spp)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    g8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    ran = torch.zeros(1, dtype=torch.int32, device="cuda")
    res = {}
    for n in (0, 32, 32):   # the first pass on the masked stream maps its queue (slow)
        ctx.set_reserved_cus(n)
        torch.cuda.synchronize()
        e0, er, eb = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(a)
        ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), g8.data_ptr(), a.cuda_stream)
        er.record(a)
        b.wait_event(e0)
        assert hooks.spt_test_blocker(ctypes.c_void_p(b.cuda_stream), 1000, 8, ctypes.c_void_p(ran.data_ptr())) == 0
        eb.record(b)
        torch.cuda.synchronize()
        res[n] = (e0.elapsed_time(er), e0.elapsed_time(eb))
        print(f"reserve {n}: render ends {res[n][0]:.2f} ms, blocker ends {res[n][1]:.2f} ms")
    ctx.close()
    assert int(ran.item()) == 8 * 3
    render_ms, blocker_ms = res[32]
    assert render_ms > 8.0, "render too short for the check"
    assert blocker_ms < 0.5 * render_ms, res
