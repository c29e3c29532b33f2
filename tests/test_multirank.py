"""CPU tests of the N>1 path: world_size-2 `gloo` processes split the frame into
interleaved strips, exchange their tiles with the same collective bench.py uses
(a gather to rank 0), and rank 0 places them with the row map.  The per-rank
tiles come from the CPU oracle (test infrastructure standing in for the GPU
render, which `test_gpu_parity.py::test_row_split_and_assemble_equals_full_frame`
covers on the device)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

W, H, SPP, B = 96, 40, 2, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_rows(rows, scene_arrays, view):
    import pyoracle as po
    sc = po.OracleScene(*scene_arrays)
    fr = po.make_frame(view, [0, 1, -3, 0], [137, 207, 240, 0], W, H, SPP, B, 1)
    tile = np.zeros((len(rows) * W, 4), np.float32)
    for k, y in enumerate(rows):
        t, _ = po.render_segment(sc, fr, int(y), int(y) + 1, 0, W)
        tile[k * W:(k + 1) * W] = t
    return tile


def _worker(rank, world, port, strip, scene_arrays, view, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import torch.distributed as dist
    from simplepathtracer_amd.distributed import FrameSplit, gather_tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        split = FrameSplit(W, H, world, strip)
        rows = split.local_rows(rank)
        tile = np.zeros((split.tile_pixels(), 4), np.float32)
        tile[:len(rows) * W] = _oracle_rows(rows, scene_arrays, view)
        local = torch.from_numpy(tile)
        gathered = torch.zeros((world * split.tile_pixels(), 4), dtype=torch.float32) if rank == 0 else None
        gather_tiles(local, gathered)
        if rank == 0:
            frame = np.zeros((H, W, 4), np.float32)
            for r in range(world):
                rr = split.local_rows(r)
                tp = split.tile_pixels()
                frame[rr] = gathered[r * tp:r * tp + len(rr) * W].numpy().reshape(len(rr), W, 4)
            q.put(frame)
    finally:
        dist.destroy_process_group()


def _bench_env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return env


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_its_own_ranks(world):
    """`bench.py --gpus N` without a launcher starts N rank processes itself (the
    driver's scaling runs call it that way); --launch-check stops after the process
    group forms, so this runs on a CPU-only host over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(_bench_env(), SPT_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--launch-check"],
                       capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
    assert line["n_gpus"] == world and line["world_size"] == world and line["backend"] == "gloo"
    assert line["ranks"] == list(range(world)) and sorted(line["local_ranks"]) == list(range(world))


def test_bench_refuses_more_ranks_than_gpus():
    """RCCL ranks need one GPU each: `--gpus N` with fewer GPUs visible exits non-zero
    instead of rendering on fewer ranks."""
    import subprocess
    import sys
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = torch.cuda.device_count() + 1
    env = dict(_bench_env(), SPT_DIST_BACKEND="nccl")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(max(n, 2))],
                       capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPUs" in r.stderr and "{" not in r.stdout


@pytest.mark.parametrize("world,strip", [(2, 8), (2, 3), (3, 4)])
def test_strip_split_gather_assemble_equals_full_frame(oracle, native, world, strip):
    import simplepathtracer_amd as spt
    from simplepathtracer_amd.distributed import FrameSplit
    split = FrameSplit(W, H, world, strip)
    owned = np.concatenate([split.local_rows(r) for r in range(world)])
    assert sorted(owned.tolist()) == list(range(H))
    scene = spt.generate_spheres(1)
    arrays = (scene.centers, scene.radii, scene.colors, scene.materials, scene.fuzz)
    view = spt.camera_basis()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, strip, arrays, view, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _oracle_rows(np.arange(H), arrays, view).reshape(H, W, 4)
    assert np.array_equal(frame.view(np.uint32), want.view(np.uint32))
