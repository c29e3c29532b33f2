"""Generate tests/golden/*.npz from the CPU restatement (oracle/).

The reference is unbuildable in this image (see oracle/spt_oracle.h), so these
vectors freeze the oracle's output: they pin the GPU path and guard the oracle
against regressions.  Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

EYE, LOOK, UP, SKY = [0, 1, -3, 0], [0, 1, 0, 0], [0, 1, 0, 0], [137, 207, 240, 0]


def cornell3():
    ref = po.init_spheres(1)
    idx = [0, 1, 2, 3]
    return po.OracleScene(ref.centers[idx], ref.radii[idx], ref.colors[idx],
                          np.array([3, 3, 1, 2], np.uint8), np.zeros(4, np.float32))


def scene_dict(sc):
    return dict(centers=sc.centers, radii=sc.radii, colors=sc.colors, materials=sc.materials, fuzz=sc.fuzz)


def main():
    view = po.camera_basis(EYE, LOOK, UP)
    out = {}
    # --- scenes (SceneGenerators.hpp), seed 1 ---
    rnd = po.generate_spheres(1)
    ref = po.init_spheres(1)
    c3 = cornell3()
    np.savez(os.path.join(HERE, "scenes.npz"), **{f"random_{k}": v for k, v in scene_dict(rnd).items()},
             **{f"reference_{k}": v for k, v in scene_dict(ref).items()},
             **{f"cornell3_{k}": v for k, v in scene_dict(c3).items()}, view=view)

    # --- config 1: 200x100, 4 spp, depth 8, full frames (RenderSegment + task) ---
    for name, sc in (("cornell3", c3), ("reference", ref)):
        fr = po.make_frame(view, EYE, SKY, 200, 100, 4, 8, 1)
        g = np.zeros(200 * 100 * 3, np.uint8)
        rgba, casts = po.render_segment(sc, fr, 0, 100, 0, 200, rgb8=g)
        out[f"c1_{name}_rgba"] = rgba
        out[f"c1_{name}_rgb8"] = g
        out[f"c1_{name}_casts"] = np.array([casts], np.uint64)
        # RenderSegmentTask on square 50x50 tiles (its colorIndex stride needs square tiles)
        gt = np.zeros(200 * 100 * 3, np.uint8)
        tiles = np.zeros((100 * 200, 4), np.float32)
        for ty in range(0, 100, 50):
            for tx in range(0, 200, 50):
                t, _ = po.render_segment(sc, fr, ty, ty + 50, tx, tx + 50, task=True, rgb8=gt)
                tiles.reshape(100, 200, 4)[ty:ty + 50, tx:tx + 50] = t.reshape(50, 50, 4)
        out[f"c1_{name}_task_rgba"] = tiles
        out[f"c1_{name}_task_rgb8"] = gt

    # --- config 2 scene, sparse pixels at 1200x800, 100 spp, depth 50 ---
    fr = po.make_frame(view, EYE, SKY, 1200, 800, 100, 50, 1)
    rng = np.random.default_rng(1234)
    px = np.stack([rng.integers(0, 1200, 48), rng.integers(0, 800, 48)], 1).astype(np.uint32)
    vals = np.zeros((len(px), 4), np.float32)
    for i, (x, y) in enumerate(px):
        v, _ = po.render_segment(rnd, fr, int(y), int(y) + 1, int(x), int(x) + 1)
        vals[i] = v[0]
    out["c2_pixels_xy"] = px
    out["c2_pixels_rgba"] = vals
    # a 16x16 window at full spp
    win, _ = po.render_segment(rnd, fr, 400, 416, 592, 608)
    out["c2_window_400_592_rgba"] = win

    # --- per-sample KATs: key, first draws, per-sample colours with cast counts ---
    keys = np.array([po.lib().spo_sample_key(1, p, s) for p, s in [(0, 0), (1, 0), (0, 1), (959999, 99)]],
                    np.uint64)
    out["kat_keys"] = keys
    import ctypes
    draws = []
    for k in keys:
        st = ctypes.c_uint64(int(k))
        draws.append([po.lib().spo_next_u32(ctypes.byref(st)) for _ in range(8)])
    out["kat_draws"] = np.array(draws, np.uint32)
    samp = np.zeros((64, 4), np.float32)
    casts = np.zeros(64, np.uint32)
    for i in range(64):
        x, y, s = (i * 37) % 1200, 300 + (i * 11) % 200, i % 100
        samp[i], casts[i] = po.trace_sample(rnd, fr, x, y, s)
    out["kat_samples_rgba"] = samp
    out["kat_samples_casts"] = casts
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
