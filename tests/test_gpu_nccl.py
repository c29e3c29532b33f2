"""GPU tests of the N > 1 frame path: the collective branch: gather_tiles with
device tensors over the nccl (= RCCL) backend -- the branch bench.py takes at N > 1 on
a node, `dist.gather` of device tiles (simplepathtracer_amd/distributed.py) -- at world
size 1 (one GPU per box), followed by rank 0's assemble kernel.  The frame and g_data
must equal a direct one-launch render bit for bit (Renderer.hpp:257-302's split,
SURVEY.md §8(e)).  The multi-rank logic itself is covered by the gloo tests
(tests/test_multirank.py)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", [0, 1])
def test_nccl_gather_then_assemble_equals_one_launch(mode):
    import torch
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as spt
    from simplepathtracer_amd.distributed import FrameSplit, gather_tiles, render_frame

    torch.cuda.set_device(0)
    own = not dist.is_initialized()
    if own:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        W, H, spp = 360, 200, 8
        ctx = spt.Context(0)
        ctx.set_scene(spt.generate_spheres(1))
        ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
        ctx.set_params(W, H, spp, 50, 1)
        stream = torch.cuda.current_stream().cuda_stream
        # the reference: one launch over the whole frame
        want = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        want8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
        ctx.render_rows_async(mode, 0, H, 1, 1, 0, 0, W, want.data_ptr(), want8.data_ptr(), stream)
        for strip in (8, 4):
            split = FrameSplit(W, H, 1, strip)
            tile = torch.zeros((split.tile_pixels(), 4), dtype=torch.float32, device="cuda")
            gathered = torch.full((split.world * split.tile_pixels(), 4), -1.0, dtype=torch.float32, device="cuda")
            frame = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
            g8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
            # bench.py's N > 1 sequence, step by step: own strips, the RCCL gather, assemble
            ctx.render_rows_async(mode, 0, H, strip, split.world, 0, 0, W, tile.data_ptr(), 0, stream)
            gather_tiles(tile, gathered)
            ctx.assemble_rows_async(gathered.data_ptr(), split.max_rows, 0, H, strip, split.world, 0, W,
                                    frame.data_ptr(), g8.data_ptr(), stream)
            torch.cuda.synchronize()
            assert torch.equal(gathered[:tile.shape[0]].view(torch.int32), tile.view(torch.int32)), strip
            assert torch.equal(frame[:, :3].contiguous().view(torch.int32), want[:, :3].contiguous().view(torch.int32)), strip
            assert torch.equal(g8, want8), strip
        # and render_frame itself (world 1 takes the one-launch path)
        frame = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        render_frame(ctx, FrameSplit(W, H, 1, 8), 0, mode, None, frame=frame, stream=stream)
        torch.cuda.synchronize()
        assert torch.equal(frame[:, :3].contiguous().view(torch.int32), want[:, :3].contiguous().view(torch.int32))
        ctx.close()
    finally:
        if own:
            dist.destroy_process_group()


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_task_ranges_assembled_equal_one_launch(parts):
    """The rank-share form of RenderSegmentTask({0, H, 0, W}) on a non-square frame
    (spt_task_range / spt_render_task_range_async, distributed.render_frame's split for it):
    each part's output range rendered alone, placed at its first output and assembled as
    one part of H rows equals the one-launch frame bit for bit, NaN outputs (bytes 0)
    included."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as spt
    from simplepathtracer_amd.renderer import task_range
    torch.cuda.set_device(0)
    W, H, spp = 360, 200, 8
    ctx = spt.Context(0)
    ctx.set_scene(spt.generate_spheres(1))
    ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
    ctx.set_params(W, H, spp, 50, 1)
    stream = torch.cuda.current_stream().cuda_stream
    want = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    want8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    ctx.render_rows_async(1, 0, H, 1, 1, 0, 0, W, want.data_ptr(), want8.data_ptr(), stream)
    stack = torch.full((W * H, 4), -7.0, dtype=torch.float32, device="cuda")
    for r in range(parts):
        a, b = task_range(W, H, parts, r)
        part = torch.full((max(b - a, 1), 4), -5.0, dtype=torch.float32, device="cuda")
        ctx.render_task_range_async(a, b, part.data_ptr(), stream)
        if b > a:
            stack[a:b].copy_(part[:b - a])
    frame = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    g8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    ctx.assemble_rows_async(stack.data_ptr(), H, 0, H, 1, 1, 0, W, frame.data_ptr(), g8.data_ptr(), stream)
    torch.cuda.synchronize()
    assert torch.equal(frame[:, :3].contiguous().view(torch.int32), want[:, :3].contiguous().view(torch.int32))
    assert torch.equal(g8, want8)
    ctx.close()

