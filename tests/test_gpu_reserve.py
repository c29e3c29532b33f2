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
    """A ~20 ms render on stream A with 32 reserved CUs (one per shader engine of each XCC:
    the mask's last bits, tools/cu_mask_probe.py); 8 blocker-shaped blocks (512 threads of
    256-VGPR waves, like RCCL's) queued on stream B just after it must all START before
    the render has ended.  An ordering of device timestamps, no ratio of times: each block
    records its start (s_memrealtime) and a one-thread kernel queued on A after the render
    records a time at which the render had ended.  How EARLY the blocks start is a timing
    property and is only printed here (without the reservation they start in the render's
    last ~1 ms, once its tail frees whole CUs; with it, at once): tools/cu_mask_probe.py
    measures it (profiles/scaling_r05.txt)."""
    import torch
    W, H, spp = 1200, 800, 400
    hooks = _hooks()
    hooks.spt_test_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hooks.spt_test_where.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    ctx = config2_ctx(spt, W, H, spp)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    g8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    nblk = 8
    res = {}
    for n in (0, 32, 32):   # the first pass on the masked stream maps its queue (slow)
        where = torch.zeros(4 * nblk, dtype=torch.int32, device="cuda")
        stamp = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctx.set_reserved_cus(n)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event()
        e0.record(a)
        ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), g8.data_ptr(), a.cuda_stream)
        assert hooks.spt_test_stamp(a.cuda_stream, stamp.data_ptr()) == 0
        b.wait_event(e0)
        assert hooks.spt_test_where(b.cuda_stream, 1000, nblk, 1, where.data_ptr()) == 0
        torch.cuda.synchronize()
        w = where.cpu().numpy().view(np.uint32).reshape(nblk, 4)
        starts = w[:, 2].astype(np.uint64) | (w[:, 3].astype(np.uint64) << np.uint64(32))
        end = np.uint64(stamp.cpu().numpy().view(np.uint64)[0])
        res[n] = (starts, end)
        late = int((starts >= end).sum())
        print(f"reserve {n}: {late} of {nblk} blocker blocks started after the render ended; "
              f"last start {(int(starts.max()) - int(end)) / 100.0:+.1f} us from the render's end")
    ctx.close()
    starts, end = res[32]
    assert (starts > 0).all()
    assert (starts < end).all(), "a blocker block waited for the render to end despite the reserved CUs"
