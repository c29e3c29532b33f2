"""Multi-GPU frame split (north_star: tile-partitioned across the GPUs of a node
with an RCCL gather of the per-tile framebuffers).

One process per GPU.  The frame's rows are dealt in interleaved `strip`-row
strips: rank r owns strips r, r+N, r+2N, ...  Each rank renders its rows into a
compact float4 tile (spt_render_rows_async); one gather over RCCL/xGMI brings
every tile to rank 0, which scatters them into the frame
and the RGB8 g_data buffer (spt_assemble_rows_async).  Per-pixel results do not
depend on the split (keyed per-(pixel, sample) RNG), so any N gives the 1-GPU frame.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .renderer import rows_count


def even_strip(height: int, world: int) -> int:
    """Rows per strip: the largest of 8, 4, 2, 1 that deals the frame's strips
    evenly over the ranks (config 2 at 8 ranks: 200 strips of 4 rows), else 8."""
    for s in (8, 4, 2, 1):
        if height % s == 0 and (height // s) % world == 0:
            return s
    return 8


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


def render_frame(ctx, split: FrameSplit, rank: int, mode: int, local_tile, gathered=None, frame=None,
                 g_data=None, stream=0, group=None, gather_events=None) -> None:
    """One distributed frame: render own rows, gather, assemble on rank 0.
    Tensors are device tensors; `stream` is the hipStream_t the launches use (the
    current torch stream: the collective follows it).  gather_events: an optional
    pair of torch.cuda.Event recorded on that stream around the gather (its time
    includes waiting for the slowest rank's render)."""
    if split.world == 1:
        ctx.render_rows_async(mode, 0, split.height, 1, 1, 0, 0, split.width,
                              frame.data_ptr() if frame is not None else 0,
                              g_data.data_ptr() if g_data is not None else 0, stream)
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
