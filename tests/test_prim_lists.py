"""Primary-ray candidate lists, checked on the CPU against the
oracle: for sampled primary rays (the oracle's own ray generation and brute-force
FindClosestIntersectionSphere, Collision.hpp:87-109, in the reference's operation order),
the closest sphere must be in the candidate list of the ray's 8x8 block and of its 8x4
block whenever that block has a list -- the property the GPU's list cast relies on for
the same winner.  The lists come from the library's host builder through
spt_prim_lists_check (no GPU).  tests/test_gpu_parity.py renders with and without them."""
import ctypes

import numpy as np
import pytest

WALK = 0xFFFFFFFF
EYE, SKY = [13.0, 2.0, 3.0, 0.0], [137.0, 207.0, 240.0, 0.0]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def prim_lists(native, centers, radii, view, eye, W, H, max_count=24):
    L = native.lib()
    n = len(radii)
    c = np.ascontiguousarray(np.asarray(centers, np.float32).reshape(n, 4))
    r = np.ascontiguousarray(np.asarray(radii, np.float32))
    v = np.ascontiguousarray(np.asarray(view, np.float32).reshape(16))
    e = np.ascontiguousarray(np.asarray(eye, np.float32).reshape(4))
    bw = (W + 7) // 8
    b8 = np.zeros(2 * bw * ((H + 7) // 8), np.uint32)
    b4 = np.zeros(2 * bw * ((H + 3) // 4), np.uint32)
    counts = np.zeros(4, np.uint32)
    assert L.spt_prim_lists_check(_p(c), _p(r), n, _p(v), _p(e), W, H, max_count, None, None, None, None, 0,
                                  _p(counts)) == 0
    cap = int(max(counts[0], counts[1]))
    ids, orig = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    assert L.spt_prim_lists_check(_p(c), _p(r), n, _p(v), _p(e), W, H, max_count, _p(b8), _p(b4), _p(ids),
                                  _p(orig), cap, _p(counts)) == 0
    assert counts[2] == bw
    return b8.reshape(-1, 2), b4.reshape(-1, 2), ids[:counts[0]], orig[:counts[1]], bool(counts[3])


def check_winners(oracle, native, scene, view, eye, W, H, spp, samples=4096, seed=1, want_on=True, focus=None):
    b8, b4, ids, orig, on = prim_lists(native, scene.centers, scene.radii, view, eye, W, H)
    assert on == want_on
    if not on:
        return 0.0, 0.0
    osc = oracle.OracleScene(scene.centers, scene.radii, scene.colors, scene.materials, scene.fuzz)
    fr = oracle.make_frame(view, eye, SKY, W, H, spp, 50, seed)
    rng = np.random.default_rng(seed)
    xs = rng.integers(0, W, samples)
    ys = rng.integers(0, H, samples)
    if focus is not None:  # half the samples inside a window (e.g. around a sphere's silhouette)
        x0, y0, x1, y1 = focus
        xs[: samples // 2] = rng.integers(x0, x1, samples // 2)
        ys[: samples // 2] = rng.integers(y0, y1, samples // 2)
    ss = rng.integers(0, spp, samples)
    win = oracle.primary_winners(osc, fr, np.stack([xs, ys, ss], 1))
    slot_of = {int(o): s for s, o in enumerate(orig) if o != WALK}
    bw = (W + 7) // 8
    listed, hits = 0, 0
    for x, y, w in zip(xs, ys, win):
        for blk in (b8[(y // 8) * bw + x // 8], b4[(y // 4) * bw + x // 8]):
            first, cnt = int(blk[0]), int(blk[1])
            if cnt == WALK:
                continue
            listed += 1
            if w < len(scene.radii):
                hits += 1
                run = ids[first:first + cnt]
                assert slot_of[int(w)] in run, f"pixel ({x}, {y}): winner {w} (slot {slot_of[int(w)]}) not in {run}"
    walk8 = float(np.mean(b8[:, 1] == WALK))
    lens = b8[b8[:, 1] != WALK, 1]
    return walk8, float(lens.mean()) if len(lens) else 0.0


@pytest.fixture(scope="module")
def spt_mod():
    import simplepathtracer_amd as spt
    return spt


def test_config2_scene_default_camera(oracle, native, spt_mod):
    scene = spt_mod.generate_spheres(1)
    view = spt_mod.camera_basis()
    walk, mean_len = check_winners(oracle, native, scene, view, spt_mod.scene.DEFAULT_EYE, 1200, 800, 100,
                                   samples=8192)
    assert walk < 0.05 and mean_len < 12  # lists for nearly every block, short ones


@pytest.mark.parametrize("eye,look", [([4.0, 1.0, 3.0, 0.0], [4.0, 1.0, 0.0, 0.0]),   # close-up of a big ball
                                      ([0.3, 0.25, 0.4, 0.0], [3.0, 0.2, 2.0, 0.0]),   # low, among the small spheres
                                      ([0.0, 30.0, 0.1, 0.0], [0.0, 0.0, 0.0, 0.0]),   # looking down
                                      ([0.0, 1.0, 0.0, 0.0], [1.0, 1.0, 0.0, 0.0])])   # inside the glass ball
def test_other_cameras(oracle, native, spt_mod, eye, look):
    scene = spt_mod.generate_spheres(1)
    view = spt_mod.camera_basis(eye, look, [0.0, 1.0, 0.0, 0.0])
    check_winners(oracle, native, scene, view, eye, 320, 200, 16, samples=6000, seed=3)


def test_silhouettes_and_ragged_frame(oracle, native, spt_mod):
    """A ragged frame (203 x 117: partial blocks at the right and bottom edges), half the
    samples in a window around the big balls' silhouettes."""
    scene = spt_mod.generate_spheres(2)
    view = spt_mod.camera_basis()
    check_winners(oracle, native, scene, view, spt_mod.scene.DEFAULT_EYE, 203, 117, 32, samples=8000, seed=5,
                  focus=(60, 30, 150, 90))


def test_stress_and_small_scenes(oracle, native, spt_mod):
    stress = spt_mod.generate_stress(3, 300)  # walked by the whole wave (fewer than 64 tree nodes)
    view = spt_mod.camera_basis()
    check_winners(oracle, native, stress, view, spt_mod.scene.DEFAULT_EYE, 256, 160, 8, samples=6000, seed=7)
    c3 = spt_mod.cornell3()
    v3 = spt_mod.camera_basis([0.0, 1.0, -3.0, 0.0], [0.0, 1.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0])
    check_winners(oracle, native, c3, v3, [0.0, 1.0, -3.0, 0.0], 200, 100, 4, samples=4000, seed=9)


def test_config5_stress_scene(oracle, native, spt_mod):
    """Config 5's 10 000-sphere stress scene at full size (the host check; the lane-walk
    kernels that render it do not use the lists); half the samples in a window over the
    grazing far field of the sphere layer."""
    stress = spt_mod.generate_stress(1, 10000)
    view = spt_mod.camera_basis()
    walk, mean_len = check_winners(oracle, native, stress, view, spt_mod.scene.DEFAULT_EYE, 1920, 1080, 256,
                                   samples=6000, seed=11, focus=(0, 380, 1920, 620))
    assert walk < 0.1 and mean_len < 16


def test_degenerate_camera_walks(oracle, native, spt_mod):
    """A non-finite view or eye turns the lists off (every block walks the tree)."""
    scene = spt_mod.generate_spheres(1)
    view = np.asarray(spt_mod.camera_basis(), np.float32).copy()
    view.reshape(16)[0] = np.inf
    check_winners(oracle, native, scene, view, spt_mod.scene.DEFAULT_EYE, 64, 64, 4, want_on=False)
    check_winners(oracle, native, scene, spt_mod.camera_basis(), [np.nan, 2.0, 3.0, 0.0], 64, 64, 4, want_on=False)


def test_threaded_build_equals_one_thread(native, monkeypatch):
    """The host builder splits large builds over threads by 64 x 64 super-block; the tables
    must be those of one thread (config 5's 10 000-sphere stress scene at 1920 x 1080)."""
    import simplepathtracer_amd as spt
    sc = spt.generate_stress(1, 10000)
    view = spt.camera_basis()
    eye = list(spt.scene.DEFAULT_EYE)
    got = []
    for th in ("1", "8"):
        monkeypatch.setenv("SPT_PRIM_THREADS", th)
        got.append(prim_lists(native, sc.centers, sc.radii, view, eye, 1920, 1080))
    for a, b in zip(got[0], got[1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
