"""Multi-GPU frame split (north_star: tile-partitioned across the GPUs of a node
with an RCCL gather of the per-tile framebuffers).

One process per GPU.  The frame's rows are dealt in interleaved `strip`-row
strips: rank r owns strips r, r+N, r+2N, ...  Each rank renders its rows into a
compact float4 tile (spt_render_rows_async); one gather over RCCL/xGMI brings
every tile to rank 0 (or the copy-engine TileTransport: peer copies from IPC
handles, ordered by stream wait/write-value packets), which scatters them into the frame
and the RGB8 g_data buffer (spt_assemble_rows_async).  Per-pixel results do not
depend on the split (keyed per-(pixel, sample) RNG), so any N gives the 1-GPU frame.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from .renderer import rows_count, task_range

MODE_TASK = 1  # spt_hip.h SPT_MODE_TASK


def even_strip(height: int, world: int) -> int:
    """Rows per strip: the tallest of 8, 4, 2 whose deal gives no rank more than 6% over an
    even share, else 1.  8-row strips keep the 8x8 pixel blocks of the primary batches and
    the candidate lists whole: at N = 8 (tools/scaling_probe.py, round 6) config 3's share
    renders in 42.85 / 46.26 / 51.05 ms with 8- / 4- / 2-row strips and config 2's at 5.9 /
    6.2 / 6.9 us per row, so config 2 at 8 ranks takes 13 or 12 strips of 8 rows (104 rows
    at most) rather than 25 of 4.  The C++ host (spt_ctx.cpp even_strip) uses the same rule."""
    if world <= 1:
        return 8
    for s in (8, 4, 2):
        strips = -(-height // s)
        rows = min(height, -(-strips // world) * s)
        if rows <= 1.06 * height / world:
            return s
    return 1


@dataclass(frozen=True)
class FrameSplit:
    width: int
    height: int
    world: int
    strip: int = 8

    @property
    def rows(self) -> list[int]:
        return [rows_count(0, self.height, self.strip, self.world, r) for r in range(self.world)]

    @property
    def max_rows(self) -> int:
        return max(self.rows)

    def local_rows(self, rank: int) -> np.ndarray:
        """Global y of each local row of `rank` (the kernel's RowMap, restated)."""
        n = rows_count(0, self.height, self.strip, self.world, rank)
        k = np.arange(n)
        blk = k // self.strip
        return (blk * self.world + rank) * self.strip + (k - blk * self.strip)

    def tile_pixels(self) -> int:
        return self.max_rows * self.width

    def aliased(self, mode: int) -> bool:
        """RenderImage's RenderSegmentTask({0, H, 0, W}) on a non-square frame aliases pixels
        across rows (TaskBasedPathTracer.hpp:103,186): the frame is then split by output
        ranges (spt_task_range) instead of row strips."""
        return mode == MODE_TASK and self.width != self.height and self.world > 1

    def task_ranges(self) -> list[tuple[int, int]]:
        return [task_range(self.width, self.height, self.world, r) for r in range(self.world)]

    def slot_pixels(self, mode: int) -> int:
        """Pixels of one rank's tile slot: its strips' rows, or its longest output range."""
        if self.aliased(mode):
            return max(b - a for a, b in self.task_ranges())
        return self.tile_pixels()


def gather_tiles(local_tile, gathered, group=None) -> None:
    """Every rank's tile -> rank 0's gathered[world*max_rows*width, 4], rank-major: one
    gather to rank 0 (RCCL send/recv pairs over xGMI), so each tile crosses one link
    once; other ranks pass gathered=None."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dst = dist.get_global_rank(group, 0) if group is not None else 0
    if local_tile.is_cuda and dist.get_backend(group) != "nccl":
        # rehearsal path (several ranks on one GPU, gloo): exchange host copies
        host = local_tile.cpu()
        parts = [host.new_empty(host.shape) for _ in range(world)] if rank == 0 else None
        dist.gather(host, parts, dst=dst, group=group)
        if rank == 0:
            for r, p in enumerate(parts):
                gathered[r * p.shape[0]:(r + 1) * p.shape[0]].copy_(p)
        return
    parts = list(gathered.chunk(world)) if rank == 0 else None
    dist.gather(local_tile, parts, dst=dst, group=group)


class TileTransport:
    """The copy-engine tile transport (spt_tiles_*, include/spt_hip.h): the alternative to
    gather_tiles' RCCL gather.  Rank 0 owns `nbuf` gathered buffers in one device
    allocation exported by IPC handle; every other rank copies its tile into its slot of
    the frame's buffer on its own stream (a device-to-device copy into peer memory, no
    collective kernel), and stream wait/write-value packets on words in a shared host
    segment order the copies, rank 0's assemble and the buffers' reuse.  Frames are
    numbered identically on every rank; frame f uses buffer f % nbuf.  Collective setup
    over `torch.distributed` (any backend: only the segment name and the 64-byte handle
    travel through it)."""

    def __init__(self, ctx, split: FrameSplit, rank: int, nbuf: int = 2, group=None, mode: int = 0):
        import os
        import secrets
        import torch.distributed as dist
        from . import _native
        self._lib = _native.lib()
        self._ctx = ctx
        self._group = group
        self.rank, self.world, self.nbuf = rank, split.world, nbuf
        self.base = 0  # frames the setup check used (verify): caller frame f is transport frame base + f
        self.tile_bytes = split.slot_pixels(mode) * 16  # float4
        src = dist.get_global_rank(group, 0) if group is not None else 0
        name = [f"{os.getpid()}_{secrets.token_hex(6)}" if rank == 0 else None]
        dist.broadcast_object_list(name, src=src, group=group)
        self._h = ctypes.c_void_p()
        # every rank runs every collective below whatever fails locally; the outcome is
        # agreed at the end (a rank that raised midway would leave the others in a barrier)
        err = []

        def attempt(fn):
            if not err:
                try:
                    fn()
                except Exception as e:  # noqa: BLE001 -- reported after the agreement
                    err.append(e)

        def create():
            _native.check(self._lib.spt_tiles_create(ctx.handle, name[0].encode(), rank, self.world,
                                                     self.tile_bytes, nbuf, ctypes.byref(self._h)), ctx.handle)

        if rank == 0:
            attempt(create)  # the segment exists before the others open it
        dist.barrier(group=group)
        if rank != 0:
            attempt(create)
        handle = [None]
        if rank == 0 and not err:
            buf = (ctypes.c_uint8 * 64)()

            def export():
                self._check(self._lib.spt_tiles_handle(self._h, buf))
                handle[0] = bytes(buf)

            attempt(export)
        dist.broadcast_object_list(handle, src=src, group=group)
        if rank != 0:
            if handle[0] is None:
                err.append(RuntimeError("rank 0 exported no buffer handle"))
            attempt(lambda: self._check(self._lib.spt_tiles_attach(
                self._h, (ctypes.c_uint8 * 64).from_buffer_copy(handle[0]))))
        dist.barrier(group=group)
        if rank == 0 and self._h.value:
            attempt(lambda: self._check(self._lib.spt_tiles_unlink(self._h)))
        oks = [None] * self.world
        dist.all_gather_object(oks, not err, group=group)
        if not all(oks):
            self.close()
            raise RuntimeError(f"tile transport setup failed on ranks {[r for r, o in enumerate(oks) if not o]}"
                               + (f": {err[0]}" if err else ""))

    def _check(self, code: int) -> None:
        from . import _native
        _native.check(code, self._ctx.handle)

    def buffer(self, frame: int) -> int:
        """Rank 0: device address of frame's gathered buffer (its own tile is slot 0)."""
        p = ctypes.c_void_p()
        self._check(self._lib.spt_tiles_buffer(self._h, self.base + frame, ctypes.byref(p)))
        return p.value

    def send(self, frame: int, d_tile: int, stream) -> None:
        """Ranks > 0: the tile at d_tile into the frame's buffer, then the ready word."""
        self._check(self._lib.spt_tiles_send_async(self._h, self.base + frame, ctypes.c_void_p(d_tile),
                                                   ctypes.c_void_p(stream)))

    def send_range(self, frame: int, d_src: int, offset: int, nbytes: int, stream) -> None:
        """Ranks > 0: nbytes at d_src to byte `offset` of the frame's buffer, then the ready word."""
        self._check(self._lib.spt_tiles_send_range_async(self._h, self.base + frame, ctypes.c_void_p(d_src), offset,
                                                         nbytes, ctypes.c_void_p(stream)))

    def recv(self, frame: int, stream) -> None:
        """Rank 0: `stream` waits for every rank's ready word of the frame."""
        self._check(self._lib.spt_tiles_recv_async(self._h, self.base + frame, ctypes.c_void_p(stream)))

    def release(self, frame: int, stream) -> None:
        """Rank 0, after its reads of the frame's buffer: the buffer's consumed word."""
        self._check(self._lib.spt_tiles_release_async(self._h, self.base + frame, ctypes.c_void_p(stream)))

    def verify(self, local_tile, stream, timeout_s: float = 20.0) -> bool:
        """Setup check (collective, before any frame): 2 x nbuf frames of a known pattern go
        through the transport -- every buffer used twice, so the consumed-word handshake runs
        -- and rank 0 compares each rank's slot with a device kernel reading the buffer (the
        assemble's access path).  A wait that does not complete within timeout_s gives the
        transport up (spt_tiles_abort unblocks every rank's streams).  True on every rank only
        if every rank saw its part complete and every slot matched; the frames used are
        skipped by later calls (self.base).  local_tile: a device float4 tensor of at least a
        slot (ranks > 0); stream: the torch.cuda.Stream the transport's packets go on."""
        import os
        import time
        import torch
        import torch.distributed as dist
        slot = self.tile_bytes // 16
        ok, checks = True, []
        with torch.cuda.stream(stream):
            for f in range(2 * self.nbuf):
                if self.rank != 0:
                    # SPT_TILES_TEST_CORRUPT=1 (tests): a wrong pattern, so the check fails
                    bad = os.environ.get("SPT_TILES_TEST_CORRUPT", "0") != "0"
                    local_tile[:slot].fill_(float(self.rank * 64 + f + 1 + (7 if bad else 0)))
                    self.send(f, local_tile.data_ptr(), stream.cuda_stream)
                else:
                    self.recv(f, stream.cuda_stream)
                    try:
                        view = torch.as_tensor(_DeviceArray(self.buffer(f), self.world * slot),
                                               device=local_tile.device)
                        for r in range(1, self.world):  # device results, read after the bounded wait
                            checks.append(view[r * slot:(r + 1) * slot].eq(float(r * 64 + f + 1)).all())
                    except Exception:  # no __cuda_array_interface__ support: no check possible
                        checks.append(False)
                    self.release(f, stream.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(stream)
                deadline = time.monotonic() + timeout_s
                while not ev.query():
                    if time.monotonic() > deadline:
                        self._lib.spt_tiles_abort(self._h)
                        ok = False
                        break
                    time.sleep(0.0005)
                if not ok:
                    break
        stream.synchronize()
        if self.rank == 0:
            ok = ok and all(bool(c) for c in checks)
        seen = [None] * self.world
        dist.all_gather_object(seen, ok, group=self._group)
        ok = all(seen)
        if not ok:
            self._lib.spt_tiles_abort(self._h)
        else:
            self.base = 2 * self.nbuf
        return ok

    def close(self) -> None:
        if self._h.value:
            self._lib.spt_tiles_destroy(self._h)
            self._h = type(self._h)()


class _DeviceArray:
    """A float4 device array at a raw address, for torch.as_tensor (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n, 4), "typestr": "<f4", "data": (ptr, False), "version": 2}


def render_frame(ctx, split: FrameSplit, rank: int, mode: int, local_tile, gathered=None, frame=None,
                 g_data=None, stream=0, group=None, gather_events=None, transport: TileTransport | None = None,
                 frame_no: int = 0) -> None:
    """One distributed frame: render own rows, gather, assemble on rank 0.
    Tensors are device tensors; `stream` is the hipStream_t the launches use (the
    current torch stream: the collective follows it).  gather_events: an optional
    pair of torch.cuda.Event recorded on that stream around the gather (its time
    includes waiting for the slowest rank's render).  transport: the copy-engine
    transport instead of the RCCL gather (frame_no: the frame's number, the same on
    every rank; rank 0 renders into its slot of the frame's buffer, `gathered` unused;
    with nbuf buffers, frames f and f + nbuf must use the same stream)."""
    if split.world == 1:
        ctx.render_rows_async(mode, 0, split.height, 1, 1, 0, 0, split.width,
                              frame.data_ptr() if frame is not None else 0,
                              g_data.data_ptr() if g_data is not None else 0, stream)
        return
    if split.aliased(mode):
        _render_frame_ranges(ctx, split, rank, local_tile, gathered, frame, g_data, stream, group, gather_events,
                             transport, frame_no)
        return
    if transport is not None:
        dst = transport.buffer(frame_no) if rank == 0 else local_tile.data_ptr()
        ctx.render_rows_async(mode, 0, split.height, split.strip, split.world, rank, 0, split.width, dst, 0, stream)
        if gather_events is not None:
            gather_events[0].record()
        if rank == 0:
            transport.recv(frame_no, stream)
        else:
            transport.send(frame_no, dst, stream)
        if gather_events is not None:
            gather_events[1].record()
        if rank == 0:
            ctx.assemble_rows_async(dst, split.max_rows, 0, split.height, split.strip, split.world, 0, split.width,
                                    frame.data_ptr() if frame is not None else 0,
                                    g_data.data_ptr() if g_data is not None else 0, stream)
            transport.release(frame_no, stream)
        return
    ctx.render_rows_async(mode, 0, split.height, split.strip, split.world, rank, 0, split.width,
                          local_tile.data_ptr(), 0, stream)
    if gather_events is not None:
        gather_events[0].record()
    gather_tiles(local_tile, gathered, group)
    if gather_events is not None:
        gather_events[1].record()
    if rank == 0:
        ctx.assemble_rows_async(gathered.data_ptr(), split.max_rows, 0, split.height, split.strip, split.world, 0,
                                split.width, frame.data_ptr() if frame is not None else 0,
                                g_data.data_ptr() if g_data is not None else 0, stream)


def _render_frame_ranges(ctx, split: FrameSplit, rank, local_tile, gathered, frame, g_data, stream, group,
                         gather_events, transport, frame_no) -> None:
    """render_frame for a non-square task-mode frame: rank r renders outputs [i0_r, i1_r)
    of the frame's row-major order (spt_render_task_range_async, the split spt_render_frame
    uses over a multi-device context); rank 0 places each range at its first output -- the
    ranges end to end are the frame -- and assembles it as one part of H rows."""
    import torch
    ranges = split.task_ranges()
    i0, i1 = ranges[rank]
    W, H = split.width, split.height

    def assemble(d_stack):
        ctx.assemble_rows_async(d_stack, H, 0, H, 1, 1, 0, W, frame.data_ptr() if frame is not None else 0,
                                g_data.data_ptr() if g_data is not None else 0, stream)

    if transport is not None:
        # the transport's buffer is the frame: rank 0 renders its range in place, the
        # others copy theirs to its offset
        dst = transport.buffer(frame_no) + 16 * i0 if rank == 0 else local_tile.data_ptr()
        ctx.render_task_range_async(i0, i1, dst, stream)
        if gather_events is not None:
            gather_events[0].record()
        if rank == 0:
            transport.recv(frame_no, stream)
        else:
            transport.send_range(frame_no, dst, 16 * i0, 16 * (i1 - i0), stream)
        if gather_events is not None:
            gather_events[1].record()
        if rank == 0:
            assemble(transport.buffer(frame_no))
            transport.release(frame_no, stream)
        return
    ctx.render_task_range_async(i0, i1, local_tile.data_ptr(), stream)
    if gather_events is not None:
        gather_events[0].record()
    gather_tiles(local_tile, gathered, group)
    if gather_events is not None:
        gather_events[1].record()
    if rank == 0:
        # slot r of the gathered stack holds range r from its start (torch's current
        # stream: the caller's, as for the gather)
        slot = local_tile.shape[0]
        stack = torch.empty((W * H, 4), dtype=torch.float32, device=gathered.device)
        for r, (a, b) in enumerate(ranges):
            if b > a:
                stack[a:b].copy_(gathered[r * slot:r * slot + (b - a)])
        assemble(stack.data_ptr())
