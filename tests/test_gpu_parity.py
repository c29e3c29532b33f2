"""GPU parity tests: the gfx950 render path (through the C ABI) against the CPU
restatement (oracle/) and the committed goldens.  Bar: bit-exact float pixels
(north_star's 1e-5 abs tolerance is below one ulp for bright pixels) and exact
RGB8 bytes.  Run on an MI355X with `pytest -m gpu`.
"""
import ctypes
import math
import threading
from fractions import Fraction

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EYE, LOOK, UP, SKY = [0, 1, -3, 0], [0, 1, 0, 0], [0, 1, 0, 0], [137, 207, 240, 0]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_bitwise(got, want, what=""):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    assert got.shape == want.shape, what
    g, w = bits(got), bits(want)
    bad = np.nonzero(g != w)
    if len(bad[0]):
        i = tuple(b[0] for b in bad)
        raise AssertionError(f"{what}: {len(bad[0])} of {g.size} lanes differ; first at {i}: "
                             f"got {got[i]!r} want {want[i]!r}")


@pytest.fixture(scope="module")
def spt():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import simplepathtracer_amd as m
    m.lib()
    return m


@pytest.fixture(scope="module")
def ctx(spt):
    c = spt.Context(0)
    yield c
    c.close()


def scene_from(spt, gs, name):
    return spt.Scene(*(gs[f"{name}_{k}"] for k in ("centers", "radii", "colors", "materials", "fuzz")))


def oscene_from(oracle, gs, name):
    return oracle.OracleScene(*(gs[f"{name}_{k}"] for k in ("centers", "radii", "colors", "materials", "fuzz")))


def setup(ctx, scene, w, h, spp, b, seed=1, view=None):
    import simplepathtracer_amd as m
    ctx.set_scene(scene)
    ctx.set_camera(m.camera_basis(EYE, LOOK, UP) if view is None else view, EYE, SKY)
    ctx.set_params(w, h, spp, b, seed)


# ---------------------------------------------------------------- numerics

def test_device_numerics_match_host(ctx, oracle):
    rng = np.random.default_rng(3)
    n = 1 << 16
    a = np.concatenate([rng.random(n - 8, dtype=np.float32) * 4,
                        np.float32([0, 1, 2, 1e-40, 255, 0.25, 3.4e38, 1e-30])])
    b = (rng.random(n, dtype=np.float32) * 3 + np.float32(1e-3)).astype(np.float32)
    u = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    u[:6] = [0, 1, 0xFFFFFF7F, 0xFFFFFF80, 0xFFFFFFFF, 0x80000000]
    out = ctx.selftest_numerics(a, b, u)
    assert_bitwise(out[:, 0], a / b, "fp32 division")
    assert_bitwise(out[:, 1], np.sqrt(a), "fp32 sqrt")
    # SampleColorRefractive's float powf / sqrtf (spt_powf.h restates glibc's powf)
    libm = ctypes.CDLL("libm.so.6")
    libm.powf.restype = ctypes.c_float
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    c_any = u.view(np.float32)
    hard = [float.fromhex(h) for h in ("0x1.003bap-24", "0x1.14708ep-1", "0x1.ef5ee8p-1", "0x1.14708ep+0")]
    for i in list(range(0, n, 7)) + [n - 8 + k for k in range(8)]:
        assert out[i, 2] == np.float32(libm.powf(float(a[i]), 5.0)), ("powf(x,5)", a[i])
        want = np.float32(libm.powf(float(c_any[i]), 5.0))
        assert out[i, 3].view(np.uint32) == want.view(np.uint32) or (np.isnan(out[i, 3]) and np.isnan(want)), \
            ("powf(any,5)", c_any[i])
        assert out[i, 4] == np.float32(libm.powf(float(a[i]), 2.0)), ("powf(x,2)", a[i])
    ha = np.float32(hard + [-0.2, 0.2] + [0] * (len(a) - len(hard) - 2))[: len(a)]
    oh = ctx.selftest_numerics(ha, b, u)
    for i in range(len(hard) + 2):
        assert oh[i, 2] == np.float32(libm.powf(float(ha[i]), 5.0)), ("hard powf", ha[i])
        assert oh[i, 4] == np.float32(libm.powf(float(ha[i]), 2.0))
    # r * sqrt(1 - c*c) < 1 and the Snell scalar r*c - sqrt(1 - r*r*(1 - c*c)), float
    r = np.float32(1.0) / np.float32(1.5)
    with np.errstate(all="ignore"):
        tir_ok = r * np.sqrt(np.float32(1) - a * a) < np.float32(1)
        k = r * a - np.sqrt(np.float32(1) - r * r * (np.float32(1) - a * a))
    same_or_nan(out[:, 5], np.where(tir_ok, k, np.float32(-1e30)), "refraction scalar")
    want_u = np.array([oracle.lib().spo_uniform_u32(int(x), -1.0, 1.0) for x in u[:4096]], np.float32)
    assert_bitwise(out[:4096, 6], want_u, "uniform(-1,1)")
    for col, lo, hi in ((12, -0.5, 0.5), (13, 0.0, 1.0)):
        want_u = np.array([oracle.lib().spo_uniform_u32(int(x), lo, hi) for x in u[:4096]], np.float32)
        assert_bitwise(out[:4096, col], want_u, f"uniform({lo},{hi})")
    assert np.array_equal(out[:, 7], np.trunc(np.where(a < 2**31, a, 0)).astype(np.int64).astype(np.uint8))
    # Normalize (Math.hpp:140-154) and c / a through the shortened division core,
    # c = any float bit pattern: NaN/inf/denormal/huge lanes take the full sequence
    c = u.view(np.float32)
    with np.errstate(all="ignore"):
        L = (a * a + b * b) + c * c
        l = np.sqrt(L)
        want = np.stack([a / l, b / l, c / l], 1)
        q = c / a
    same_or_nan(out[:, 8:11], want, "Normalize")
    same_or_nan(out[:, 11], q, "division over the full float range")
    # the fold's rebuild of a diffuse sample: j halvings one by one (a denormal result
    # rounds at every step), as the render loop applied them (SingleThreadPathTracer.hpp:31)
    j = ((u.astype(np.uint64) * 2654435761) & 0xFFFFFFFF) >> 23
    j = (j % 301).astype(np.int64)
    hc, ha = c.copy(), a.copy()
    with np.errstate(all="ignore"):
        for k in range(301):
            hc = np.where(k < j, hc * np.float32(0.5), hc).astype(np.float32)
            ha = np.where(k < j, ha * np.float32(0.5), ha).astype(np.float32)
    same_or_nan(out[:, 14], hc, "halvings over the full float range")
    same_or_nan(out[:, 15], ha, "halvings")


def same_or_nan(got, want, what):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    nan = np.isnan(got) & np.isnan(want)
    bad = (got.view(np.uint32) != want.view(np.uint32)) & ~nan
    assert not bad.any(), f"{what}: {int(bad.sum())} mismatches, first {got[bad][:4]} vs {want[bad][:4]}"


# ---------------------------------------------------------------- goldens

@pytest.mark.parametrize("name", ["cornell3", "reference"])
def test_config1_frame_matches_golden(spt, ctx, golden, golden_scenes, name):
    setup(ctx, scene_from(spt, golden_scenes, name), 200, 100, 4, 8)
    g = np.zeros(200 * 100 * 3, np.uint8)
    rgba = ctx.render_segment(0, 100, 0, 200, g)
    assert_bitwise(rgba[:, :3], golden[f"c1_{name}_rgba"][:, :3], f"C1 {name} float pixels")
    assert np.array_equal(g, golden[f"c1_{name}_rgb8"])
    st = ctx.stats()
    assert st["samples"] >= 200 * 100 * 4


@pytest.mark.parametrize("name", ["cornell3", "reference"])
def test_config1_task_tiles_match_golden(spt, ctx, golden, golden_scenes, name):
    setup(ctx, scene_from(spt, golden_scenes, name), 200, 100, 4, 8)
    g = np.zeros(200 * 100 * 3, np.uint8)
    out = np.zeros((100, 200, 4), np.float32)
    for ty in range(0, 100, 50):
        for tx in range(0, 200, 50):
            t = ctx.render_segment(ty, ty + 50, tx, tx + 50, g, task=True)
            out[ty:ty + 50, tx:tx + 50] = t.reshape(50, 50, 4)
    assert_bitwise(out.reshape(-1, 4)[:, :3], golden[f"c1_{name}_task_rgba"][:, :3], "C1 task")
    assert np.array_equal(g, golden[f"c1_{name}_task_rgb8"])


def test_config2_sparse_pixels_and_window_match_golden(spt, ctx, golden, golden_scenes):
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 100, 50)
    win = ctx.render_segment(400, 416, 592, 608)
    assert_bitwise(win[:, :3], golden["c2_window_400_592_rgba"][:, :3], "C2 window")
    for (x, y), want in zip(golden["c2_pixels_xy"], golden["c2_pixels_rgba"]):
        got = ctx.render_segment(int(y), int(y) + 1, int(x), int(x) + 1)
        assert_bitwise(got[0, :3], want[:3], f"C2 pixel {(x, y)}")


# ---------------------------------------------------------------- vs live oracle

def test_per_sample_colours_and_cast_counts(spt, ctx, oracle, golden_scenes):
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 12, 50, seed=77)
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, 1200, 800, 12, 50, 77)
    yB, yE, xB, xE = 350, 358, 500, 540
    ctx.reset_stats()
    samp = ctx.render_samples(yB, yE, xB, xE, 12)
    casts = 0
    for p in range(samp.shape[0]):
        y, x = yB + p // (xE - xB), xB + p % (xE - xB)
        for s in range(12):
            want, c = oracle.trace_sample(sc, fr, x, y, s)
            casts += c
            assert_bitwise(samp[p, s, :3], want[:3], f"sample {(x, y, s)}")
    assert ctx.stats()["casts"] == casts


@pytest.mark.parametrize("task", [False, True])
def test_region_vs_oracle_with_gdata_bytes(spt, ctx, oracle, golden_scenes, task):
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 8, 50, seed=5)
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, 1200, 800, 8, 50, 5)
    g = np.full(1200 * 800 * 3, 0xAB, np.uint8)
    gw = g.copy()
    yB, xB, t = 300, 610, 32
    got = ctx.render_segment(yB, yB + t, xB, xB + t, g, task=task)
    want, _ = oracle.render_segment(sc, fr, yB, yB + t, xB, xB + t, task=task, rgb8=gw)
    assert_bitwise(got[:, :3], want[:, :3], "region")
    assert np.array_equal(g, gw), "g_data bytes (region written, rest untouched)"


def _mirror_lattice():
    """6x6x6 lattice of fuzzy mirror spheres over the ground: ~4% of paths need
    more than RenderSegmentTask's 10 passes (TaskBasedPathTracer.hpp:81)."""
    pts = [[(i - 2.5), 0.2 + j, 1.5 + k, 0] for i in range(6) for j in range(6) for k in range(6)]
    c = np.float32([[0, -1000.5, 0, 0]] + pts)
    n = len(c)
    r = np.float32([1000] + [0.47] * (n - 1))
    col = np.float32([[30, 144, 255, 0]] + [[200, 100, 50, 0]] * (n - 1))
    m = np.uint8([3] + [1] * (n - 1))
    fz = np.float32([0] + [0.02] * (n - 1))
    return c, r, col, m, fz


def test_task_mode_drops_deep_specular_paths(spt, ctx, oracle):
    arrays = _mirror_lattice()
    setup(ctx, spt.Scene(*arrays), 64, 64, 16, 8, seed=9)
    ctx.reset_stats()
    got = ctx.render_segment(0, 64, 0, 64, task=True)
    assert ctx.stats()["dropped"] > 0
    osc = oracle.OracleScene(*arrays)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 64, 64, 16, 8, 9)
    want, _ = oracle.render_segment(osc, fr, 0, 64, 0, 64, task=True)
    assert_bitwise(got[:, :3], want[:, :3], "task mode with drops")
    got_seg = ctx.render_segment(0, 64, 0, 64, task=False)
    want_seg, _ = oracle.render_segment(osc, fr, 0, 64, 0, 64)
    assert_bitwise(got_seg[:, :3], want_seg[:, :3], "segment mode, deep specular chains")


def _mirror_glass_lattice():
    """The mirror lattice with every other sphere glass: paths of one sample finish
    in different RenderSegmentTask passes and queues (TaskBasedPathTracer.hpp:81-193)."""
    c, r, col, m, fz = _mirror_lattice()
    m = m.copy()
    m[2::2] = 2
    return c, r, col, m, fz


def same_bits_or_nan(got, want, what):
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    nan = np.isnan(got) & np.isnan(want)
    bad = (bits(got) != bits(want)) & ~nan
    assert not bad.any(), f"{what}: {int(bad.sum())} lanes differ, first got {got[bad][:3]} want {want[bad][:3]}"


@pytest.mark.parametrize("scene_name,y0,x0,w,h", [("random", 200, 300, 300, 200), ("random", 300, 500, 40, 90),
                                                   ("lattice", 0, 0, 96, 20), ("lattice", 8, 4, 30, 50)])
def test_task_mode_non_square_tiles_alias_like_the_reference(spt, ctx, oracle, golden_scenes, scene_name, y0, x0, w, h):
    """RenderSegmentTask on a non-square tile strides colorIndex rows by segmentHeight
    (TaskBasedPathTracer.hpp:103,186): pixel (p % W, p / W) gets colors[p], the sum of
    every tile pixel (dx, dy) with dx + dy * H == p, added within each sample in the
    reference's breadth-first order (pass, diffuse before skybox, queue order);
    indices no pixel maps to resolve to 0 * (1/0) = NaN.  Config 2's own tiling
    (1200x800, tc = 4) is 300x200; 96x20 has five sources per index."""
    if scene_name == "random":
        arrays = [golden_scenes[f"random_{k}"] for k in ("centers", "radii", "colors", "materials", "fuzz")]
        view, fw, fh, spp, b, seed = golden_scenes["view"], 1200, 800, 3, 50, 4
    else:
        arrays = list(_mirror_glass_lattice())
        view, fw, fh, spp, b, seed = spt.camera_basis(EYE, LOOK, UP), 128, 64, 12, 8, 9
    setup(ctx, spt.Scene(*arrays), fw, fh, spp, b, seed=seed, view=view)
    g = np.full(fw * fh * 3, 0xAB, np.uint8)
    gw = g.copy()
    got = ctx.render_segment(y0, y0 + h, x0, x0 + w, g, task=True)
    fr = oracle.make_frame(view, EYE, SKY, fw, fh, spp, b, seed)
    want, _ = oracle.render_segment(oracle.OracleScene(*arrays), fr, y0, y0 + h, x0, x0 + w, task=True, rgb8=gw)
    same_bits_or_nan(got[:, :3], want[:, :3], f"task mode, {w}x{h} tile")
    assert np.isnan(want[:, 0]).any() == (w != h)
    assert np.array_equal(g, gw), "g_data bytes"


# ---------------------------------------------------------------- edge cases

def test_empty_region_is_a_noop(spt, ctx, golden_scenes):
    setup(ctx, scene_from(spt, golden_scenes, "reference"), 16, 16, 2, 3)
    g = np.full(16 * 16 * 3, 7, np.uint8)
    out = ctx.render_segment(5, 5, 0, 16, g)
    assert out.size == 0 and (g == 7).all()


def test_zero_spheres_is_all_sky(spt, ctx, oracle):
    e = np.zeros((0, 4), np.float32)
    scene = spt.Scene(e, np.zeros(0, np.float32), e, np.zeros(0, np.uint8), np.zeros(0, np.float32))
    setup(ctx, scene, 24, 12, 3, 4)
    got = ctx.render_segment(0, 12, 0, 24)
    osc = oracle.OracleScene(e, np.zeros(0, np.float32), e, np.zeros(0, np.uint8), np.zeros(0, np.float32))
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 24, 12, 3, 4, 1)
    want, casts = oracle.render_segment(osc, fr, 0, 12, 0, 24)
    assert casts == 24 * 12 * 3
    assert_bitwise(got[:, :3], want[:, :3], "sky only")


def test_skybox_material_and_single_bounce(spt, ctx, oracle, golden_scenes):
    """Material SKYBOX on a sphere falls through to the sky (SingleThreadPathTracer.hpp:98-111)."""
    gs = golden_scenes
    m = gs["reference_materials"].copy()
    m[5] = 0
    m[7] = 7  # unknown id behaves like SKYBOX too
    scene = spt.Scene(gs["reference_centers"], gs["reference_radii"], gs["reference_colors"], m,
                      gs["reference_fuzz"])
    setup(ctx, scene, 40, 40, 5, 1)
    got = ctx.render_segment(0, 40, 0, 40)
    osc = oracle.OracleScene(gs["reference_centers"], gs["reference_radii"], gs["reference_colors"], m,
                             gs["reference_fuzz"])
    fr = oracle.make_frame(gs["view"], EYE, SKY, 40, 40, 5, 1, 1)
    want, _ = oracle.render_segment(osc, fr, 0, 40, 0, 40)
    assert_bitwise(got[:, :3], want[:, :3], "skybox material / bounces=1")


def test_more_than_255_spheres(spt, ctx, oracle):
    """Extension beyond the reference's uint8 index (Collision.hpp:87-92); pinned
    against the oracle's uint32 restatement only (the reference hangs)."""
    s = spt.generate_stress(11, 300)
    setup(ctx, s, 96, 64, 4, 10)
    got = ctx.render_segment(20, 44, 30, 62)
    osc = oracle.OracleScene(s.centers, s.radii, s.colors, s.materials, s.fuzz)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 96, 64, 4, 10, 1)
    want, _ = oracle.render_segment(osc, fr, 20, 44, 30, 62)
    assert_bitwise(got[:, :3], want[:, :3], "300 spheres")


def test_diffuse_codes_saturate_where_albedos_vanish(spt, ctx, oracle, golden_scenes):
    """Sample codes saturate j at min(bounces - 1, jz), jz = the halvings after which every
    finite albedo is 0 (spt_internal.h diffuse_code): tiny, denormal and infinite albedos at
    depth 40, where jz (~30) is below bounces - 1 and halve_n takes its denormal path."""
    gs = golden_scenes
    col = gs["reference_colors"].copy()
    col[:, :3] *= np.float32(1e-37)
    col[1, :3] = np.float32([1e-44, 3e-42, 7e-40])  # denormal albedos
    col[3, 1] = np.float32(np.inf)
    scene = spt.Scene(gs["reference_centers"], gs["reference_radii"], col, gs["reference_materials"],
                      gs["reference_fuzz"])
    setup(ctx, scene, 48, 32, 6, 40)
    got = ctx.render_segment(0, 32, 0, 48)
    osc = oracle.OracleScene(gs["reference_centers"], gs["reference_radii"], col, gs["reference_materials"],
                             gs["reference_fuzz"])
    fr = oracle.make_frame(gs["view"], EYE, SKY, 48, 32, 6, 40, 1)
    want, _ = oracle.render_segment(osc, fr, 0, 32, 0, 48)
    same_bits_or_nan(got[:, :3], want[:, :3], "saturated diffuse codes")
    assert (got[:, :3] != 0).any() and np.isinf(got[:, 1]).any()


def test_scene_beyond_four_million_slots(spt, oracle, golden_scenes):
    """Sample codes are 2 + j * slots + slot (the former 22 slot bits refused
    scenes over 4 194 304 slots).  4.3 M tiny spheres far behind the camera, then the
    reference scene's 10, so every hit lands on a slot above 2^22; brute force (cluster
    size 0) keeps the host build cheap."""
    gs = golden_scenes
    n_far = 4_300_000
    far = np.zeros((n_far, 4), np.float32)
    far[:, 0] = np.arange(n_far, dtype=np.float32) * np.float32(1e-3)
    far[:, 2] = np.float32(-500.0)
    c = np.concatenate([far, gs["reference_centers"]]).astype(np.float32)
    r = np.concatenate([np.full(n_far, 1e-3, np.float32), gs["reference_radii"]]).astype(np.float32)
    col = np.concatenate([np.full((n_far, 4), 9, np.float32), gs["reference_colors"]]).astype(np.float32)
    m = np.concatenate([np.full(n_far, 3, np.uint8), gs["reference_materials"]]).astype(np.uint8)
    f = np.concatenate([np.zeros(n_far, np.float32), gs["reference_fuzz"]]).astype(np.float32)
    cx = spt.Context(0)
    try:
        cx.set_cluster_size(0)
        setup(cx, spt.Scene(c, r, col, m, f), 64, 48, 2, 6)
        got = cx.render_segment(20, 24, 28, 36)
    finally:
        cx.close()
    osc = oracle.OracleScene(c, r, col, m, f)
    fr = oracle.make_frame(gs["view"], EYE, SKY, 64, 48, 2, 6, 1)
    want, _ = oracle.render_segment(osc, fr, 20, 24, 28, 36)
    assert_bitwise(got[:, :3], want[:, :3], "4.3 M sphere slots")


def test_nondefault_camera_and_odd_frame(spt, ctx, oracle, golden_scenes):
    view = spt.camera_basis([2, 3, -4, 0], [0, 0.5, 2, 0], UP)
    setup(ctx, scene_from(spt, golden_scenes, "random"), 131, 77, 3, 12, seed=3, view=view)
    got = ctx.render_segment(10, 50, 7, 120)
    osc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(view, EYE, SKY, 131, 77, 3, 12, 3)
    want, _ = oracle.render_segment(osc, fr, 10, 50, 7, 120)
    assert_bitwise(got[:, :3], want[:, :3], "camera")


def test_invalid_arguments_raise(spt, ctx, golden_scenes):
    setup(ctx, scene_from(spt, golden_scenes, "reference"), 16, 16, 2, 3)
    with pytest.raises(spt.SptError):
        ctx.set_params(16, 16, 2, 0, 1)  # bounces = 0
    with pytest.raises(spt.SptError):
        ctx.set_params(16, 16, 0, 3, 1)  # spp = 0
    with pytest.raises(spt.SptError):
        ctx.render_segment(0, 17, 0, 16)  # outside the frame
    bad = np.eye(4, dtype=np.float32).ravel()
    with pytest.raises(spt.SptError):
        ctx.set_camera(bad, EYE, SKY)  # viewMatrix row 3 must be zero


# ---------------------------------------------------------------- full-size properties

@pytest.mark.parametrize("task", [False, True])
def test_workspace_batches_fold_in_order(spt, ctx, golden_scenes, task):
    """Several sample batches (odd ones on the companion stream, double-buffered) fold in
    batch order: bit-identical to one batch; again on a caller stream of its own."""
    import torch
    def render(*r):
        return ctx.render_segment(*r, task=task)

    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 10, 50, seed=4)
    a = render(200, 264, 100, 228)
    ctx.set_workspace(64 * 128 * (8 if task else 4) * 3)  # 3 samples per batch: 4 batches (4- / 8-byte slots)
    b = render(200, 264, 100, 228)
    ctx.reset_stats()
    st = torch.cuda.Stream()
    out = torch.zeros((64 * 128, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill runs on the current stream, the render on st
    ctx.render_rows_async(spt.MODE_TASK if task else spt.MODE_SEGMENT, 200, 264, 1, 1, 0, 100, 228,
                          out.data_ptr(), 0, st.cuda_stream)
    st.synchronize()
    launches = ctx.stats()["launches"]
    ctx.set_workspace(4 << 30)
    assert_bitwise(b, a, "batched vs single-batch")
    assert_bitwise(out.cpu().numpy(), a, "batched on a caller stream vs single-batch")
    assert launches == 4


def test_row_split_and_assemble_equals_full_frame(spt, ctx, golden_scenes):
    import torch
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 4, 50, seed=2)
    full = torch.zeros((800 * 1200, 4), dtype=torch.float32, device="cuda")
    g_full = torch.zeros(1200 * 800 * 3, dtype=torch.uint8, device="cuda")
    ctx.render_rows_async(0, 0, 800, 1, 1, 0, 0, 1200, full.data_ptr(), g_full.data_ptr())
    ctx.synchronize()
    parts, strip = 3, 8
    rows = [spt.rows_count(0, 800, strip, parts, p) for p in range(parts)]
    mr = max(rows)
    tiles = torch.zeros((parts, mr * 1200, 4), dtype=torch.float32, device="cuda")
    for p in range(parts):
        ctx.render_rows_async(0, 0, 800, strip, parts, p, 0, 1200, tiles[p].data_ptr(), 0)
    frame = torch.zeros_like(full)
    g = torch.zeros_like(g_full)
    ctx.assemble_rows_async(tiles.data_ptr(), mr, 0, 800, strip, parts, 0, 1200, frame.data_ptr(), g.data_ptr())
    ctx.synchronize()
    assert torch.equal(frame.view(torch.int32), full.view(torch.int32))
    assert torch.equal(g, g_full)


def test_config2_every_pixel_vs_oracle(spt, ctx, oracle, golden_scenes):
    """The whole config-2 frame (1200x800, the box-tree default traversal) at 4 spp,
    every pixel's float RGB and g_data bytes against the oracle's
    RenderImageParallelMain (16x16 tiles, 16 threads); and RenderImage's
    RenderSegmentTask over the whole non-square frame (colorIndex aliasing across the
    frame) at 1 spp against the oracle's single-rectangle task render."""
    W, H = 1200, 800
    sc = oscene_from(oracle, golden_scenes, "random")
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, 4, 50, seed=11)
    g = np.zeros(W * H * 3, np.uint8)
    got = ctx.render_segment(0, H, 0, W, g)
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, 4, 50, 11)
    want, want8 = oracle.render_image_parallel(sc, fr, 16, mode=0)
    assert_bitwise(got[:, :3], want[:, :3], "config 2, every pixel, 4 spp")
    assert np.array_equal(g, want8)
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, 1, 50, seed=12)
    g = np.zeros(W * H * 3, np.uint8)
    got = ctx.render_segment(0, H, 0, W, g, task=True)
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, 1, 50, 12)
    g_want = np.zeros_like(g)
    want, _ = oracle.render_segment(sc, fr, 0, H, 0, W, task=True, rgb8=g_want)
    same_or_nan(got[:, :3], want[:, :3], "RenderImage (task mode, whole non-square frame)")
    assert np.array_equal(g, g_want)


def test_config2_full_frame_properties(spt, ctx, oracle, golden_scenes):
    """BASELINE config 2 at full size: every sample accounted for, deterministic,
    and random pixels bit-exact vs the oracle."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 100, 50)
    ctx.reset_stats()
    g1 = np.zeros(1200 * 800 * 3, np.uint8)
    a = ctx.render_segment(0, 800, 0, 1200, g1)
    st = ctx.stats()
    assert st["samples"] == 1200 * 800 * 100
    assert 1.5 < st["casts"] / st["samples"] < 4.0
    b = ctx.render_segment(0, 800, 0, 1200)
    assert_bitwise(a, b, "determinism")
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, 1200, 800, 100, 50, 1)
    rng = np.random.default_rng(99)
    for _ in range(24):
        x, y = int(rng.integers(0, 1200)), int(rng.integers(0, 800))
        want, _ = oracle.render_segment(sc, fr, y, y + 1, x, x + 1)
        assert_bitwise(a[y * 1200 + x, :3], want[0, :3], f"pixel {(x, y)}")
    assert np.isfinite(a[:, :3]).all()


def test_concurrent_render_jobs_share_a_context(spt, golden_scenes):
    """RenderImageParallelMain (Renderer.hpp:257-302) calls the entry point from
    several threads at once on disjoint tiles."""
    g = spt.Globals(scene_from(spt, golden_scenes, "random"), width=240, height=160, samples=6, bounces=50)
    spt.RenderImageParallelMain(g, thread_count=4)
    tiled = g.g_data.copy()
    g.g_data[:] = 0
    spt.RenderSegment(spt.RenderSegmentData(0, 160, 0, 240), g)
    assert np.array_equal(tiled, g.g_data)
    g.ctx.close()


@pytest.mark.parametrize("w,h,tc,task,devices", [(1200, 800, 4, 0, None), (1200, 800, 4, 1, None),
                                                  (1200, 800, 8, 0, "0,0"), (320, 160, 16, 0, None),
                                                  (320, 160, 16, 1, None), (1200, 800, 4, 0, "svc"),
                                                  (1200, 800, 4, 1, "svc")])
def test_cpp_dropin_shim_renders_like_the_context(spt, golden_scenes, tmp_path, w, h, tc, task, devices):
    """The C++ RenderSegment/RenderSegmentTask shim, driven by RenderJob-style
    concurrent threads over a tc x tc tile grid (config 2's 300x200 tiles at tc = 4,
    non-square: task mode aliases; 256 tiles of 20x10 at tc = 16, batched many to a
    launch), writes the same g_data bytes as tile renders through the context (its
    page-locked g_data written in place by the batched fold); SPT_DEVICES spreads the
    tiles over a multi-device context; SPT_SERVICE=1 makes them service jobs (with repeated
    frames, so the read-ahead serves them too)."""
    import os
    import subprocess
    from test_abi import _build_shim_harness
    exe = _build_shim_harness(tmp_path)
    out = tmp_path / "g_data.bin"
    env = dict(os.environ)
    frames = []
    if devices == "svc":
        # the shim's calls as jobs of the render service (SPT_SERVICE=1), three more frames:
        # the tiling read-ahead arms after the first and serves the others through it
        env["SPT_SERVICE"] = "1"
        frames = ["3"]
    elif devices:
        env["SPT_DEVICES"] = devices
    subprocess.run([exe, str(out), str(w), str(h), "6", "50", str(tc), str(task)] + frames, check=True, timeout=300,
                   env=env)
    got = np.fromfile(out, np.uint8)
    c = spt.Context(0)
    setup(c, scene_from(spt, golden_scenes, "random"), w, h, 6, 50)
    want = np.zeros(w * h * 3, np.uint8)
    sw, sh = w // tc, h // tc
    for j in range(tc):
        for i in range(tc):
            c.render_segment(sh * j, sh * j + sh, sw * i, sw * i + sw, want, task=bool(task))
    c.close()
    bad = np.nonzero(got != want)[0]
    px = bad // 3
    tiles = sorted(set(zip(((h - 1 - px // w) // sh).tolist(), ((px % w) // sw).tolist())))
    assert bad.size == 0, f"{bad.size} bytes differ in tiles (row, col) {tiles[:24]} (of {len(tiles)})"


@pytest.mark.parametrize("service,transport,world,mode,config", [
    (0, "rccl", 2, "segment", "c2"), (1, "rccl", 2, "segment", "c2"), (0, "ipc", 2, "segment", "c2"),
    (1, "ipc", 2, "segment", "c2"), (0, "rccl", 3, "task", "c2"), (0, "ipc", 3, "task", "c2"),
    (1, "rccl", 3, "task", "c2"), (1, "ipc", 3, "task", "c2"), (0, "ipc", 2, "segment", "c5"),
    (0, "rccl", 2, "task", "c2w"), (0, "ipc", 2, "segment", "c3"), (1, "auto", 2, "segment", "c2"),
    (1, "auto-fail", 2, "segment", "c2"), (0, "ipc", 2, "task", "c2+wavefront")])
def test_bench_two_ranks_on_one_gpu_matches_one_rank(spt, tmp_path, service, transport, world, mode, config):
    """bench.py's N>1 flow (strip split, gather to rank 0, rank-0 assemble)
    rehearsed with two gloo ranks sharing cuda:0, launched by bench.py itself
    (`--gpus 2`, no torchrun): the line says 2 ranks and g_data equals N=1's.
    service=1 runs the N>1 default of a real node -- every rank share a job of the
    rank's resident render service, gathered per frame (bench.py `use_svc`) -- with each
    rank's session on half its grid (SPT_SVC_GRID_DIV=2) so both ranks' sessions are
    resident on the one GPU.  transport="ipc": the copy-engine TileTransport instead of
    the gather (rank 1's copies into rank 0's IPC-exported buffers, stream wait/write
    packets on shared host words), over enough frames that each of the two gathered
    buffers is reused (its consumed word gates the next copy); also three ranks in task
    mode, whose non-square frame aliases pixels across rows (TaskBasedPathTracer.hpp:103,
    186): split by output ranges (spt_task_range), gathered and placed end to end; and
    config 5's LDS-tree scene (1920 x 1080 x 256 spp) over the transport, and the
    ~500-sphere scene (its 89-node tree takes the LDS lane walk) in task mode, and config 3
    (3840 x 2160 x 1024 spp: each rank share rendered in sample batches) over the transport;
    the default (--transport auto: the copy-engine transport once its setup check passes)
    and its fallback to the RCCL-path gather when the check fails (a corrupted pattern);
    the wavefront engine's rank shares in task mode."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    one, two = tmp_path / "one.bin", tmp_path / "two.bin"
    base = [sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
            "--no-dropin", "--mode", mode, "--config", config.split("+")[0]]
    if "+" in config:  # the render engine: "+wavefront" = the material-queue variant
        base += ["--engine", config.split("+")[1]]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    subprocess.run(base + ["--dump", str(one)], check=True, timeout=300, cwd=root, env=env)
    env["SPT_DIST_BACKEND"] = "gloo"
    extra = []
    if service:
        env["SPT_SVC_GRID_DIV"] = str(world)
        extra = ["--service", "1", "--steps", "3", "--warmup", "1"]
    if transport != "rccl":
        extra = ["--service", str(service), "--steps", "5", "--warmup", "2"]
    if transport == "auto-fail":
        env["SPT_TILES_TEST_CORRUPT"] = "1"  # the setup check fails: bench falls back to RCCL
    extra += ["--transport", transport.split("-")[0]]
    r = subprocess.run(base + ["--gpus", str(world), "--dump", str(two)] + extra, check=True, timeout=300, cwd=root,
                       env=env, capture_output=True, text=True)
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
    assert line["n_gpus"] == world and line["world_size"] == world and line["backend"] == "gloo"
    assert line["config"]["render_service"] == bool(service)
    want = {"rccl": ("rccl", None), "ipc": ("ipc", "passed"), "auto": ("ipc", "passed"),
            "auto-fail": ("rccl", "failed")}[transport]
    assert (line["config"]["transport"], line["config"]["transport_check"]) == want
    # the session leaves a block slot free only beside the copy-engine transport
    assert line["config"]["service_full_grid"] == (bool(service) and want[0] == "rccl")
    assert len(line["ranks"]["render_ms"]) == world and min(line["ranks"]["render_ms"]) > 0
    a, b = np.fromfile(one, np.uint8), np.fromfile(two, np.uint8)
    W, H = {"c5": (1920, 1080), "c3": (3840, 2160)}.get(config.split("+")[0], (1200, 800))
    assert a.size == b.size == W * H * 3
    bad = np.nonzero(a != b)[0]
    rows = np.unique(H - 1 - (bad // 3) // W)  # g_data row r holds image row y = H-1-r
    assert bad.size == 0, f"{bad.size} bytes differ in {rows.size} rows, first rows {rows[:16]}, a={a[bad[:6]]} b={b[bad[:6]]}"


@pytest.mark.parametrize("scene_name", ["random", "stress"])
def test_culling_is_exact(spt, ctx, golden_scenes, scene_name):
    """Cluster-tree culling (spt_accel.cpp) skips only spheres that cannot pass:
    frames and ray counts are bit-identical to brute force (cluster size 0) for
    any cluster size and tree shape (flat lists of 4- and 8-slot leaves, binary,
    4-ary, 16-ary trees)."""
    if scene_name == "random":
        scene, W, H, spp, region = scene_from(spt, golden_scenes, "random"), 1200, 800, 16, (0, 800, 0, 1200)
    else:
        scene, W, H, spp, region = spt.generate_stress(5, 2000), 480, 270, 8, (0, 270, 0, 480)
    setup(ctx, scene, W, H, spp, 50)
    outs = []
    for k, b in ((0, 0), (8, 0), (4, 0), (3, 0), (8, 2), (8, 4), (3, 16), (5, 4)):
        ctx.set_cluster_size(k)
        ctx.set_cluster_tree(b)
        ctx.reset_stats()
        outs.append(((k, b), ctx.render_segment(*region), ctx.stats()["casts"]))
    ctx.set_cluster_size(spt._native.CLUSTER_AUTO)
    ctx.set_cluster_tree(spt._native.TREE_AUTO)
    for kb, img, casts in outs[1:]:
        assert_bitwise(img, outs[0][1], f"cluster size / tree branching {kb} vs brute force")
        assert casts == outs[0][2]
    with pytest.raises(spt.SptError):
        ctx.set_cluster_size(9)  # clusters hold at most kClusterSlots = 8 members
    with pytest.raises(spt.SptError):
        ctx.set_cluster_tree(1)


@pytest.mark.parametrize("shift,scale", [((3000.0, 0.0, -2000.0), 1.0), ((0.0, 0.0, 0.0), 1e-3),
                                         ((-40.0, 7.0, 55.0), 30.0)])
def test_culling_is_exact_far_and_scaled(spt, ctx, golden_scenes, shift, scale):
    """The conservative node and member pretests carry margins that
    grow with |C| + |o|; a scene translated far from the origin, shrunk to the scale
    of the 1e-3 thresholds, or enlarged still renders bit-identically to brute force
    (flat lists of 4-slot leaves and trees)."""
    base = scene_from(spt, golden_scenes, "random")
    c = np.array(base.centers, np.float32).copy()
    c[:, :3] = (c[:, :3] * np.float32(scale) + np.float32(shift)).astype(np.float32)
    scene = spt.Scene(c, (np.asarray(base.radii, np.float32) * np.float32(scale)).astype(np.float32),
                      base.colors, base.materials, base.fuzz)
    eye = [(e * scale + s) for e, s in zip(EYE[:3], shift)] + [0]
    look = [(e * scale + s) for e, s in zip(LOOK[:3], shift)] + [0]
    view = spt.camera_basis(eye, look, UP)
    ctx.set_scene(scene)
    ctx.set_camera(view, eye, SKY)
    ctx.set_params(320, 200, 8, 50, 3)
    outs = []
    for k, b in ((0, 0), (spt._native.CLUSTER_AUTO, spt._native.TREE_AUTO), (8, 4)):
        ctx.set_cluster_size(k)
        ctx.set_cluster_tree(b)
        ctx.reset_stats()
        outs.append(((k, b), ctx.render_segment(0, 200, 0, 320), ctx.stats()["casts"]))
    ctx.set_cluster_size(spt._native.CLUSTER_AUTO)
    ctx.set_cluster_tree(spt._native.TREE_AUTO)
    for kb, img, casts in outs[1:]:
        assert_bitwise(img, outs[0][1], f"shift {shift} scale {scale}, culling {kb} vs brute force")
        assert casts == outs[0][2]


@pytest.mark.parametrize("n", [1500, 15000])
@pytest.mark.parametrize("case", ["ties", "far", "small", "large"])
def test_lane_walk_is_exact(spt, ctx, case, n):
    """The lane walk of the box tree (find_closest_lane: each lane its own path and
    leaves, per-lane tie-break by original index) from LDS (1 500
    spheres: the 1 024-thread kernel) and from global memory (15 000: the 256-thread
    render_kernel_glane) on a stress scene: with every small sphere duplicated (exact
    distance ties: the lower index wins, as in the reference's strict scan), moved 3600
    units from the origin, shrunk 1000x and enlarged 30x.  Frames and ray counts equal
    brute force."""
    base = spt.generate_stress(7, n)
    c, r = np.asarray(base.centers, np.float32).copy(), np.asarray(base.radii, np.float32).copy()
    col, m, f = np.asarray(base.colors, np.float32), np.asarray(base.materials), np.asarray(base.fuzz, np.float32)
    shift, scale = (0.0, 0.0, 0.0), 1.0
    if case == "ties":
        small = np.nonzero(r < 0.5)[0]
        col2 = col[small].copy()
        col2[:, :3] = 255.0 - col2[:, :3]
        m2 = np.where(m[small] == 3, 1, 3).astype(m.dtype)
        c, r = np.concatenate([c, c[small]]), np.concatenate([r, r[small]])
        col, m, f = np.concatenate([col, col2]), np.concatenate([m, m2]), np.concatenate([f, f[small]])
    else:
        shift, scale = {"far": ((3000.0, 0.0, -2000.0), 1.0), "small": ((0.0, 0.0, 0.0), 1e-3),
                        "large": ((-40.0, 7.0, 55.0), 30.0)}[case]
        c[:, :3] = (c[:, :3] * np.float32(scale) + np.float32(shift)).astype(np.float32)
        r = (r * np.float32(scale)).astype(np.float32)
    scene = spt.Scene(c, r, col, m, f)
    eye = [(e * scale + s) for e, s in zip(EYE[:3], shift)] + [0]
    look = [(e * scale + s) for e, s in zip(LOOK[:3], shift)] + [0]
    ctx.set_scene(scene)
    ctx.set_camera(spt.camera_basis(eye, look, UP), eye, SKY)
    ctx.set_params(320, 200, 4, 50, 5)
    outs = []
    for k, b in ((0, 0), (spt._native.CLUSTER_AUTO, spt._native.TREE_AUTO), (8, 4)):
        ctx.set_cluster_size(k)
        ctx.set_cluster_tree(b)
        ctx.reset_stats()
        img = ctx.render_segment(0, 200, 0, 320)
        st = ctx.stats()
        if k != 0:
            assert st["block_threads"] == (1024 if n == 1500 else 256), (k, b, st["block_threads"])
        outs.append(((k, b), img, st["casts"]))
    ctx.set_cluster_size(spt._native.CLUSTER_AUTO)
    ctx.set_cluster_tree(spt._native.TREE_AUTO)
    for kb, img, casts in outs[1:]:
        assert_bitwise(img, outs[0][1], f"lane walk {case}, culling {kb} vs brute force")
        assert casts == outs[0][2]


@pytest.mark.parametrize("task", [False, True])
def test_progressive_passes_equal_lower_spp_renders(spt, ctx, golden_scenes, task):
    """spt_render_progressive (the preview of RenderImageParallelMain): after every pass
    the outputs are the render at the samples done so far, bit for bit, and the last
    pass is the full render; a callback can stop it early."""
    scene, W, H = scene_from(spt, golden_scenes, "random"), 160, 96
    region = (10, 70, 20, 140)
    seen = []
    setup(ctx, scene, W, H, 20, 50)
    g = np.zeros(W * H * 3, np.uint8)
    snaps = {}

    def cb(done):
        seen.append(done)
        snaps[done] = g.copy()

    full = ctx.render_progressive(*region, 7, g, cb, task=task)
    assert seen == [7, 14, 20]
    for m in (7, 14):
        setup(ctx, scene, W, H, m, 50)
        gm = np.zeros_like(g)
        ctx.render_segment(*region, gm, task=task)
        assert np.array_equal(snaps[m], gm), f"preview after {m} samples"
    setup(ctx, scene, W, H, 20, 50)
    g2 = np.zeros_like(g)
    assert_bitwise(full, ctx.render_segment(*region, g2, task=task), "final pass vs one-shot render")
    assert np.array_equal(g, g2)
    stopped = []
    part = ctx.render_progressive(*region, 5, None, lambda d: stopped.append(d) or d >= 10, task=task)
    assert stopped == [5, 10]
    setup(ctx, scene, W, H, 10, 50)
    assert_bitwise(part, ctx.render_segment(*region, task=task), "stopped after 10 samples")
    setup(ctx, scene, W, H, 20, 50)


def test_pinned_gdata_renders_the_same(spt, ctx, golden_scenes):
    """spt_pin_host page-locks the caller's g_data (the per-frame UpdateTexture source,
    Renderer.hpp:157-164); renders into it are unchanged."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), 120, 80, 6, 50)
    g_plain = np.zeros(120 * 80 * 3, np.uint8)
    a = ctx.render_segment(0, 80, 0, 120, g_plain)
    g_pin = np.zeros_like(g_plain)
    ctx.pin_host(g_pin)
    ctx.pin_host(g_pin)  # idempotent
    b = ctx.render_segment(0, 80, 0, 120, g_pin)
    ctx.unpin_host(g_pin)
    assert_bitwise(a, b, "pinned vs pageable")
    assert np.array_equal(g_plain, g_pin)
    with pytest.raises(spt.SptError):
        ctx.unpin_host(g_pin)


def test_config5_scene_region_vs_oracle(spt, ctx, oracle):
    """BASELINE config 5's 10 000-sphere scene (cluster tree with line / front / near
    culling): a 48x24 region of the 1920x1080 frame at 8 spp,
    depth 50, every pixel bit-exact against the oracle's brute-force uint32 scan
    (parity unpinned against the reference itself, which hangs past 255 spheres)."""
    s = spt.generate_stress(1, 10000)
    setup(ctx, s, 1920, 1080, 8, 50)
    region = (600, 624, 900, 948)
    got = ctx.render_segment(*region)
    osc = oracle.OracleScene(s.centers, s.radii, s.colors, s.materials, s.fuzz)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 1920, 1080, 8, 50, 1)
    want, _ = oracle.render_segment(osc, fr, *region)
    assert_bitwise(got[:, :3], want[:, :3], "config-5 scene region")


@pytest.mark.parametrize("n", [10000, 20000, 60000])
def test_tree_kernels_lds_and_scalar_vs_oracle(spt, ctx, oracle, n):
    """The three tree walks: up to 2431 nodes each lane walks layout 0
    from the block's LDS copy (render_kernel_lds); up to 9000 nodes (20 000 spheres)
    from global memory (render_kernel_glane); a 60 000-sphere tree is walked by the
    whole wave with scalar loads over the 8 octant layouts.  A 16x8 region at 4 spp
    through the batched drop-in path and the device-resident path, bit-exact against
    the oracle's brute-force scan, and the same ray count."""
    import ctypes
    s = spt.generate_stress(3, n)
    c = np.ascontiguousarray(s.centers, np.float32)
    r = np.ascontiguousarray(s.radii, np.float32)
    nodes = ctypes.c_uint32(0)
    P = ctypes.c_void_p
    assert spt.lib().spt_accel_check(c.ctypes.data_as(P), r.ctypes.data_as(P), len(r), 8, 3,
                                            ctypes.byref(nodes)) == 0
    want_walk = {10000: "lds", 20000: "global", 60000: "wave"}[n]
    walk = "lds" if nodes.value + 1 <= 2432 else "global" if nodes.value <= 9000 else "wave"
    assert walk == want_walk, nodes.value
    setup(ctx, s, 1920, 1080, 4, 50)
    region = (500, 508, 944, 960)
    ctx.reset_stats()
    got = ctx.render_segment(*region)
    osc = oracle.OracleScene(s.centers, s.radii, s.colors, s.materials, s.fuzz)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, 1920, 1080, 4, 50, 1)
    want, casts = oracle.render_segment(osc, fr, *region)
    assert_bitwise(got[:, :3], want[:, :3], f"{n}-sphere region")
    assert ctx.stats()["casts"] == casts
    # the device-resident path (spt_render_rows_async: the unbatched kernels)
    import torch
    yB, yE, xB, xE = region
    d = torch.zeros(((yE - yB) * (xE - xB), 4), dtype=torch.float32, device="cuda")
    ctx.render_rows_async(0, yB, yE, 1, 1, 0, xB, xE, d.data_ptr(), 0)
    ctx.synchronize()
    assert_bitwise(d.cpu().numpy()[:, :3], want[:, :3], f"{n}-sphere region, device-resident")


def test_config3_full_frame_batches_vs_oracle(spt, ctx, oracle, golden_scenes):
    """BASELINE config 3 at full size (3840x2160, 1024 spp, depth 50): 6 sample batches
    of the workspace folded in order; sampled pixels bit-exact against the oracle and
    the RGB8 bytes of those pixels equal WritePixel of the oracle's colour."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), 3840, 2160, 1024, 50)
    ctx.reset_stats()
    g = np.zeros(3840 * 2160 * 3, np.uint8)
    a = ctx.render_segment(0, 2160, 0, 3840, g)
    st = ctx.stats()
    assert st["samples"] == 3840 * 2160 * 1024 and st["launches"] > 1
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, 3840, 2160, 1024, 50, 1)
    rng = np.random.default_rng(7)
    for _ in range(6):
        x, y = int(rng.integers(0, 3840)), int(rng.integers(0, 2160))
        gw = np.zeros(3840 * 2160 * 3, np.uint8)
        want, _ = oracle.render_segment(sc, fr, y, y + 1, x, x + 1, rgb8=gw)
        assert_bitwise(a[y * 3840 + x, :3], want[0, :3], f"pixel {(x, y)}")
        i = 3 * ((2160 - 1 - y) * 3840 + x)
        assert np.array_equal(g[i:i + 3], gw[i:i + 3])


# ---------------------------------------------------------------- multi-device context

@pytest.mark.parametrize("devices,task,W,H", [([0, 0], False, 360, 200), ([0, 0, 0], False, 360, 200),
                                             ([0, 0], True, 360, 200), ([0, 0, 0], True, 360, 200),
                                             ([0, 0, 0], True, 96, 250), ([0, 0], True, 64, 64)])
def test_multi_device_frame_equals_one_device(spt, golden_scenes, devices, task, W, H):
    """spt_render_frame over a device list (one process driving
    several GPUs; here device 0 listed several times): interleaved strips per member,
    peer-copy gather to member 0, assemble -- bit-identical to a one-device frame.  Task
    mode on a non-square frame (RenderImage's aliased RenderSegmentTask) is split by
    colorIndex ranges instead (wide and tall frames; NaN pixels where no source maps)."""
    spp = 6
    one = spt.Context(0)
    setup(one, scene_from(spt, golden_scenes, "random"), W, H, spp, 50)
    g1 = np.zeros(W * H * 3, np.uint8)
    want = one.render_frame(g1, task=task)
    ref = one.render_segment(0, H, 0, W, task=task)
    one.close()
    same_bits_or_nan(want, ref, "one-device render_frame vs render_segment")
    multi = spt.Context(devices=devices)
    setup(multi, scene_from(spt, golden_scenes, "random"), W, H, spp, 50)
    multi.reset_stats()
    gm = np.zeros_like(g1)
    got = multi.render_frame(gm, task=task)
    st = multi.stats()
    multi.close()
    same_bits_or_nan(got[:, :3], want[:, :3], f"{len(devices)} members")
    assert np.array_equal(gm, g1)
    if task and W != H:
        # a member whose colorIndex range no pixel maps into only writes NaN (no render)
        assert 1 <= st["launches"] <= len(devices)
        # each member renders the rows holding its colorIndex range's sources (a tall
        # frame's rows dy >= W hold none: dx + dy H >= W H is never resolved)
        assert 0 < st["samples"] <= 2 * W * H * spp
    else:
        assert st["launches"] == len(devices) and st["samples"] == W * H * spp


@pytest.mark.parametrize("scene_kind,task", [("stress", False), ("stress", True), ("random500", True)])
def test_batched_concurrent_calls_on_lane_walk_scenes(spt, scene_kind, task):
    """RenderImageParallelMain's concurrent calls (Renderer.hpp:257-302) batched into one
    launch per batch (spt_batch.cpp) on scenes whose tree takes the LDS lane walk -- the
    10 000-sphere stress scene (render_kernel_lds_batch, 1 024-thread blocks) and the
    ~500-sphere one -- in both modes (task mode on its non-square tiles aliases): the same
    g_data bytes as one call per tile in turn, and every call took the batch path (how
    many share one launch depends on when the threads' calls arrive: at 4 spp a tile can
    finish before the next call, so the count is not asserted)."""
    scene = spt.generate_stress(5, 10000) if scene_kind == "stress" else spt.generate_spheres(1, z_end=37.5)
    W, H = 320, 180
    g = spt.Globals(scene, width=W, height=H, samples=4, bounces=50)
    g.ctx.reset_stats()
    spt.RenderImageParallelMain(g, thread_count=4, task=task)
    got = g.g_data.copy()
    st = g.ctx.stats()
    assert st["batched_calls"] == 16 and 1 <= st["batches"] <= 16
    tiles = spt.Globals(scene, width=W, height=H, samples=4, bounces=50, context=g.ctx)
    fn = spt.RenderSegmentTask if task else spt.RenderSegment
    for j in range(4):
        for i in range(4):
            fn(spt.MakeRenderSegmentData(i, j, W // 4, H // 4, tiles), tiles)
    assert np.array_equal(got, tiles.g_data)
    g.ctx.close()


def test_multi_device_context_serves_render_jobs(spt, golden_scenes):
    """RenderImageParallelMain's concurrent RenderJob tiles (Renderer.hpp:257-302) on a
    two-member context: tiles go to the least busy member, same g_data bytes."""
    g = spt.Globals(scene_from(spt, golden_scenes, "random"), width=240, height=160, samples=6, bounces=50)
    spt.RenderSegment(spt.RenderSegmentData(0, 160, 0, 240), g)
    want = g.g_data.copy()
    g.ctx.close()
    g2 = spt.Globals(scene_from(spt, golden_scenes, "random"), width=240, height=160, samples=6, bounces=50,
                     devices=[0, 0])
    spt.RenderImageParallelMain(g2, thread_count=8)
    assert np.array_equal(g2.g_data, want)
    g2.ctx.close()


def test_progress_callback_may_call_into_the_context(spt, ctx, golden_scenes):
    """The progress callback runs with the context unlocked (no self-deadlock): stats()
    works from it, while a setter of the same context is refused (SPT_ERR_STATE)."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), 64, 48, 8, 50)
    seen, errs = [], []

    def cb(done):
        seen.append(ctx.stats()["samples"])
        try:
            ctx.set_params(64, 48, 8, 50, 2)
        except spt.SptError as e:
            errs.append(e.code)

    ctx.reset_stats()
    ctx.render_progressive(0, 48, 0, 64, 4, None, cb)
    assert seen == [64 * 48 * 4, 64 * 48 * 8]
    assert errs == [2, 2]


def test_concurrent_tiles_overlap_and_match(spt, ctx, golden_scenes):
    """16 RenderJob-style threads on one context (their calls batched into shared
    launches); bytes equal the serial render."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), 320, 160, 4, 50)
    want = np.zeros(320 * 160 * 3, np.uint8)
    ctx.render_segment(0, 160, 0, 320, want)
    got = np.zeros_like(want)
    tiles = [(y, y + 40, x, x + 80) for y in range(0, 160, 40) for x in range(0, 320, 80)]
    errors = []

    def job(t):
        try:
            ctx.render_segment(*t, got)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=job, args=(t,)) for t in tiles]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    assert np.array_equal(got, want)


@pytest.mark.parametrize("task", [False, True])
def test_batched_calls_match_single_calls(spt, golden_scenes, monkeypatch, task):
    """Concurrent spt_render_segment[_task] calls are rendered in batches (one render
    and one fold launch over a table of rectangles, spt_batch.cpp render_batched): float
    pixels and g_data bytes of every tile equal the same calls rendered one by one
    without batching (SPT_BATCH=0), for square and non-square tiles (task mode: the
    colorIndex aliasing per tile) and ragged sizes; the stats count every call."""
    scene = scene_from(spt, golden_scenes, "random")
    W, H, spp = 330, 170, 3
    tiles = [(0, 40, 0, 100), (0, 40, 100, 140), (40, 170, 0, 33), (40, 97, 33, 330), (97, 170, 33, 200),
             (97, 170, 200, 330), (0, 40, 140, 330)]
    n_part = len(tiles)  # a partition of the frame: these write g_data
    tiles = tiles + [(y, y + 13, x, x + 13) for y, x in ((150, 10), (0, 300), (60, 60))]  # overlapping repeats
    monkeypatch.setenv("SPT_BATCH", "0")
    ref = spt.Context(0)
    monkeypatch.delenv("SPT_BATCH")
    setup(ref, scene, W, H, spp, 50)
    want8 = np.zeros(W * H * 3, np.uint8)
    want = [ref.render_segment(*t, want8 if k < n_part else None, task=task) for k, t in enumerate(tiles)]
    assert ref.stats()["batches"] == 0
    ref.close()
    c = spt.Context(0)
    setup(c, scene, W, H, spp, 50)
    c.reset_stats()
    got8 = np.zeros_like(want8)
    got = [None] * len(tiles)
    errors = []
    go = threading.Barrier(len(tiles))

    def job(k):
        try:
            go.wait()
            got[k] = c.render_segment(*tiles[k], got8 if k < n_part else None, task=task)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=job, args=(k,)) for k in range(len(tiles))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    st = c.stats()
    c.close()
    assert not errors
    for k, t in enumerate(tiles):
        assert_bitwise(got[k], want[k], f"tile {t}")
    assert np.array_equal(got8, want8)
    assert st["batched_calls"] == len(tiles) and 1 <= st["batches"] <= len(tiles)
    assert st["launches"] == st["batches"]


# ---------------------------------------------------------------- configs 4 and 5 at full size

def test_config4_eight_way_strip_split_equals_one_part(spt, ctx, golden_scenes):
    """BASELINE config 4's split (3840x2160, the config-2 scene, 8 parts of
    even_strip(2160, 8) = 8-row interleaved strips, tiles gathered and assembled) rehearsed
    on one GPU at 2 spp: bit-identical to the 1-part frame.  Both paths: the device
    API (rows + assemble, what each bench rank runs) and spt_render_frame over an
    8-member context (the C++ host's multi-device path)."""
    import torch
    from simplepathtracer_amd.distributed import even_strip
    W, H, spp, parts = 3840, 2160, 2, 8
    strip = even_strip(H, parts)
    # 270 eight-row strips: 34 for parts 0-5, 33 for parts 6-7 (ragged tiles, padded slots)
    assert strip == 8
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, spp, 50, seed=3)
    full = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    g_full = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, full.data_ptr(), g_full.data_ptr())
    ctx.synchronize()
    rows = [spt.rows_count(0, H, strip, parts, p) for p in range(parts)]
    assert rows == [272] * 6 + [264] * 2 and sum(rows) == H
    tiles = torch.full((parts, max(rows) * W, 4), -3.0, dtype=torch.float32, device="cuda")
    for p in range(parts):
        ctx.render_rows_async(0, 0, H, strip, parts, p, 0, W, tiles[p].data_ptr(), 0)
    frame = torch.zeros_like(full)
    g = torch.zeros_like(g_full)
    ctx.assemble_rows_async(tiles.data_ptr(), max(rows), 0, H, strip, parts, 0, W, frame.data_ptr(), g.data_ptr())
    ctx.synchronize()
    assert torch.equal(frame.view(torch.int32), full.view(torch.int32))
    assert torch.equal(g, g_full)
    multi = spt.Context(devices=[0] * parts)
    setup(multi, scene_from(spt, golden_scenes, "random"), W, H, spp, 50, seed=3)
    gm = np.zeros(W * H * 3, np.uint8)
    fm = multi.render_frame(gm)
    multi.close()
    assert np.array_equal(fm.view(np.int32), full.cpu().numpy().view(np.int32))
    assert np.array_equal(gm, g_full.cpu().numpy())


def test_config4_full_spp_split_equals_config3_frame(spt, ctx, oracle, golden_scenes):
    """BASELINE config 4 at its own size and depth (3840x2160, 1024 spp, depth 50): the 8
    rank shares of the interleaved 8-row strips (what each of 8 bench ranks renders; one
    launch each, 1.06 G samples), assembled as rank 0 does after the gather, equal the
    one-GPU config-3 frame bit for bit, and sampled pixels equal the oracle.  The RCCL
    gather itself needs 8 GPUs (tests/test_multirank.py covers its logic over gloo)."""
    import torch
    from simplepathtracer_amd.distributed import even_strip
    W, H, spp, parts = 3840, 2160, 1024, 8
    strip = even_strip(H, parts)
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, spp, 50)
    full = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    g_full = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, full.data_ptr(), g_full.data_ptr())
    rows = spt.rows_count(0, H, strip, parts, 0)
    tiles = torch.zeros((parts, rows * W, 4), dtype=torch.float32, device="cuda")
    ctx.reset_stats()
    for p in range(parts):
        ctx.render_rows_async(0, 0, H, strip, parts, p, 0, W, tiles[p].data_ptr(), 0)
    frame = torch.zeros_like(full)
    g = torch.zeros_like(g_full)
    ctx.assemble_rows_async(tiles.data_ptr(), rows, 0, H, strip, parts, 0, W, frame.data_ptr(), g.data_ptr())
    ctx.synchronize()
    st = ctx.stats()
    assert st["samples"] == W * H * spp
    assert torch.equal(frame.view(torch.int32), full.view(torch.int32))
    assert torch.equal(g, g_full)
    a = frame.cpu().numpy()
    g8 = g.cpu().numpy()
    sc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(golden_scenes["view"], EYE, SKY, W, H, spp, 50, 1)
    rng = np.random.default_rng(11)
    for _ in range(4):
        x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
        gw = np.zeros(W * H * 3, np.uint8)
        want, _ = oracle.render_segment(sc, fr, y, y + 1, x, x + 1, rgb8=gw)
        assert_bitwise(a[y * W + x, :3], want[0, :3], f"C4 pixel {(x, y)}")
        i = 3 * ((H - 1 - y) * W + x)
        assert np.array_equal(g8[i:i + 3], gw[i:i + 3])


def test_culling_is_exact_with_exact_distance_ties(spt, ctx, golden_scenes):
    """Every small sphere of the config-2 scene duplicated (same centre and radius,
    another colour and material, a higher index): each hit is an exact distance tie,
    which the reference's strict '>' scan gives to the lower index.  The box tree
    (near test: strict, so ties are never culled) and the flat list keep that winner:
    frames and ray counts equal brute force."""
    base = scene_from(spt, golden_scenes, "random")
    c, r = np.asarray(base.centers, np.float32), np.asarray(base.radii, np.float32)
    col, m, f = np.asarray(base.colors, np.float32), np.asarray(base.materials), np.asarray(base.fuzz, np.float32)
    small = np.nonzero(r < 0.5)[0]
    col2 = col[small].copy()
    col2[:, :3] = 255.0 - col2[:, :3]
    m2 = np.where(m[small] == 3, 1, 3).astype(m.dtype)  # diffuse <-> mirror
    scene = spt.Scene(np.concatenate([c, c[small]]), np.concatenate([r, r[small]]), np.concatenate([col, col2]),
                      np.concatenate([m, m2]), np.concatenate([f, f[small]]))
    setup(ctx, scene, 320, 200, 8, 50, seed=4)
    outs = []
    for k, b in ((0, 0), (spt._native.CLUSTER_AUTO, spt._native.TREE_AUTO), (4, 0), (8, 2)):
        ctx.set_cluster_size(k)
        ctx.set_cluster_tree(b)
        ctx.reset_stats()
        outs.append(((k, b), ctx.render_segment(0, 200, 0, 320), ctx.stats()["casts"]))
    ctx.set_cluster_size(spt._native.CLUSTER_AUTO)
    ctx.set_cluster_tree(spt._native.TREE_AUTO)
    for kb, img, casts in outs[1:]:
        assert_bitwise(img, outs[0][1], f"duplicated spheres, culling {kb} vs brute force")
        assert casts == outs[0][2]


def test_config5_box_tree_equals_brute_force(spt, ctx):
    """The config-5 scene (10 000 spheres in a flat layer: the grazing rays the box
    margins exist for) over the whole 1920x1080 frame at 2 spp, rendered through the box tree
    walked from LDS, through the scalar-load walk of the octant layouts (a 2-ary tree
    of 8-sphere clusters has more than the LDS kernel's 2 431 nodes) and brute force
    (every sphere tested for every ray, the reference's scan): the same float bits and
    the same ray count."""
    s = spt.generate_stress(1, 10000)
    W, H = 1920, 1080
    setup(ctx, s, W, H, 2, 50, seed=21)
    outs = []
    for k, b in ((spt._native.CLUSTER_AUTO, spt._native.TREE_AUTO), (8, 2), (0, 0)):
        ctx.set_cluster_size(k)
        ctx.set_cluster_tree(b)
        ctx.reset_stats()
        outs.append(((k, b), ctx.render_segment(0, H, 0, W), ctx.stats()))
    ctx.set_cluster_size(spt._native.CLUSTER_AUTO)
    ctx.set_cluster_tree(spt._native.TREE_AUTO)
    assert outs[0][2]["block_threads"] == 1024 and outs[1][2]["block_threads"] == 256  # LDS / scalar walk
    for kb, img, st in outs[:2]:
        assert_bitwise(img, outs[2][1], f"config 5 scene, culling {kb} vs brute force")
        assert st["casts"] == outs[2][2]["casts"]


def test_config5_full_frame_properties(spt, ctx, oracle):
    """BASELINE config 5 at full size (10 000 spheres, 1920x1080, 256 spp, depth 50,
    LDS tree kernel): every sample accounted for, deterministic, and sampled pixels
    bit-exact vs the oracle's brute-force uint32 scan."""
    s = spt.generate_stress(1, 10000)
    W, H, spp = 1920, 1080, 256
    setup(ctx, s, W, H, spp, 50)
    ctx.reset_stats()
    a = ctx.render_segment(0, H, 0, W)
    st = ctx.stats()
    assert st["samples"] == W * H * spp
    assert 1.0 < st["casts"] / st["samples"] < 8.0
    assert np.isfinite(a[:, :3]).all()
    b = ctx.render_segment(0, H, 0, W)
    assert_bitwise(a, b, "determinism")
    osc = oracle.OracleScene(s.centers, s.radii, s.colors, s.materials, s.fuzz)
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, W, H, spp, 50, 1)
    rng = np.random.default_rng(5)
    for _ in range(6):
        x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
        want, _ = oracle.render_segment(osc, fr, y, y + 1, x, x + 1)
        assert_bitwise(a[y * W + x, :3], want[0, :3], f"pixel {(x, y)}")


@pytest.mark.parametrize("task", [False, True])
def test_claim_queues_render_the_same(spt, golden_scenes, monkeypatch, task):
    """Claims come from one counter per XCD (RenderArgs::n_queues, spt_kernels.hip
    claim_next): 1, 3 and 8 queues give bit-identical frames and count every sample,
    on a full region, on launches with fewer claims than queues (the trailing queues
    are empty) and through the batched drop-in path."""
    scene = scene_from(spt, golden_scenes, "random")
    regions = [(0, 120, 0, 200), (37, 45, 90, 98), (5, 6, 7, 8)]
    out = {}
    for q in ("1", "3", "8"):
        monkeypatch.setenv("SPT_QUEUES", q)
        c = spt.Context(0)
        setup(c, scene, 200, 120, 5, 50, seed=3)
        c.reset_stats()
        out[q] = [c.render_segment(*r, task=task) for r in regions]
        st = c.stats()
        got8 = np.zeros(200 * 120 * 3, np.uint8)
        tiles = [(y, y + 40, x, x + 50) for y in range(0, 120, 40) for x in range(0, 200, 50)]
        th = [threading.Thread(target=c.render_segment, args=(*t, got8), kwargs={"task": task}) for t in tiles]
        for t in th:
            t.start()
        for t in th:
            t.join()
        out[q].append(got8)
        c.close()
        if not task:
            assert st["samples"] == 5 * sum((r[1] - r[0]) * (r[3] - r[2]) for r in regions)
    monkeypatch.delenv("SPT_QUEUES")
    for q in ("3", "8"):
        for k, (a, b) in enumerate(zip(out[q], out["1"])):
            assert_bitwise(a, b, f"queues {q} vs 1, part {k}")


def test_small_launches_on_two_streams_render_the_same(spt, ctx, golden_scenes):
    """Frames in flight on two streams (the bench's rank shares): a launch of under 3 Ki
    items per wave takes the smaller grid (spt_ctx.cpp render_grid, grid_small).  The
    strips of an 8-way split rendered alternately on two streams, the same strips on the
    caller's stream alone, and the whole frame assembled from either, are bit-identical."""
    import torch
    setup(ctx, scene_from(spt, golden_scenes, "random"), 1200, 800, 4, 50, seed=5)
    parts, strip = 8, 4
    rows = [spt.rows_count(0, 800, strip, parts, p) for p in range(parts)]
    mr = max(rows)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    two = torch.zeros((parts, mr * 1200, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill runs on the current stream, the renders on others
    for p in range(parts):
        ctx.render_rows_async(0, 0, 800, strip, parts, p, 0, 1200, two[p].data_ptr(), 0, streams[p % 2].cuda_stream)
    torch.cuda.synchronize()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert ctx.stats()["grid_blocks"] <= 5 * ncu, "the small-launch grid was not taken"
    one = torch.zeros_like(two)
    for p in range(parts):
        ctx.render_rows_async(0, 0, 800, strip, parts, p, 0, 1200, one[p].data_ptr(), 0)
    ctx.synchronize()
    assert torch.equal(two.view(torch.int32), one.view(torch.int32))
    full = torch.zeros((800 * 1200, 4), dtype=torch.float32, device="cuda")
    ctx.render_rows_async(0, 0, 800, 1, 1, 0, 0, 1200, full.data_ptr(), 0)
    frame = torch.zeros_like(full)
    ctx.assemble_rows_async(two.data_ptr(), mr, 0, 800, strip, parts, 0, 1200, frame.data_ptr(), 0)
    ctx.synchronize()
    assert torch.equal(frame.view(torch.int32), full.view(torch.int32))


def _render_variants(spt, golden_scenes, view, eye, W, H, spp):
    """Outputs of one context for the list tests: full frame (segment, task), a rank share
    of interleaved 4-row strips, a batched drop-in tile, two service jobs; and ray counts."""
    import torch
    c = spt.Context(0)
    c.set_scene(scene_from(spt, golden_scenes, "random"))
    c.set_camera(view, eye, SKY)
    c.set_params(W, H, spp, 50, 4)
    out, casts = {}, []
    for name, (mode, strip, parts, part) in {"seg": (0, 1, 1, 0), "task": (1, 1, 1, 0), "share": (0, 4, 8, 3)}.items():
        n = spt.rows_count(0, H, strip, parts, part) * W
        rgba = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
        g8 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
        c.reset_stats()
        c.render_rows_async(mode, 0, H, strip, parts, part, 0, W, rgba.data_ptr(), g8.data_ptr() if parts == 1 else 0)
        c.synchronize()
        out[name] = (rgba.cpu().numpy(), g8.cpu().numpy())
        casts.append(c.stats()["casts"])
    g = np.zeros(W * H * 3, np.uint8)
    c.reset_stats()
    out["tile"] = (c.render_segment(H // 3, H // 3 + 37, W // 5, W // 5 + 61, g_data=g), g)
    casts.append(c.stats()["casts"])
    c.service_start()
    jobs = []
    for k in range(2):
        rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        c.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), 0)
        jobs.append(rgba)
    c.service_stop()
    c.synchronize()
    out["svc"] = (jobs[0].cpu().numpy(), jobs[1].cpu().numpy())
    st = c.stats()
    c.close()
    return out, casts, st


@pytest.mark.parametrize("case", ["default", "closeup", "low", "inside", "ragged"])
def test_primary_lists_equal_tree_walk(spt, golden_scenes, monkeypatch, case):
    """Primary batches cast against their block's candidate list (DESIGN.md §4.2 item 6,
    spt_path.h prim_list_cast): frames, ray counts and g_data bytes equal the tree walk's
    (SPT_PRIM_LISTS=0) -- full frames in both modes, a rank share of 4-row strips (its
    8x8 tiles span two 8x4 blocks: union of lists), a batched drop-in tile and service
    jobs -- for the default camera, a close-up of a big ball, a low view among the small
    spheres, an eye inside the glass ball, and a ragged 203 x 117 frame."""
    cams = {"default": (EYE, LOOK), "closeup": ([4.0, 1.0, 3.0, 0.0], [4.0, 1.0, 0.0, 0.0]),
            "low": ([0.3, 0.25, 0.4, 0.0], [3.0, 0.2, 2.0, 0.0]), "inside": ([0.0, 1.0, 0.0, 0.0], [1.0, 1.0, 0.0, 0.0]),
            "ragged": (EYE, LOOK)}
    eye, look = cams[case]
    W, H = (203, 117) if case == "ragged" else (320, 200)
    view = spt.camera_basis(eye, look, UP)
    got, casts, st = _render_variants(spt, golden_scenes, view, eye, W, H, 8)
    assert st["prim_list_blocks"] > 0
    monkeypatch.setenv("SPT_PRIM_LISTS", "0")
    want, casts0, st0 = _render_variants(spt, golden_scenes, view, eye, W, H, 8)
    assert st0["prim_list_blocks"] == 0
    for k in want:
        assert_bitwise(got[k][0], want[k][0], f"{case} {k}")
        assert np.array_equal(got[k][1], want[k][1]), f"{case} {k}: second output differs"
    assert casts == casts0


@pytest.mark.parametrize("W,H,y0,y1,x0,x1", [(70000, 4, 0, 4, 65504, 65600), (70000, 4, 0, 4, 69936, 70000),
                                              (4, 70000, 65520, 65560, 0, 4), (4, 70000, 69980, 70000, 0, 4)])
def test_frames_of_65536_or_more_columns_or_rows(spt, ctx, oracle, golden_scenes, W, H, y0, y1, x0, x1):
    """A primary batch packs its lanes' pixels as (y << 16 | x) for the candidate-list lookup
    (spt_path.h prim_list_cast): frames of 65 536 or more columns or rows have no
    lists (the batches walk the tree) and render like the oracle past column / row 65 535."""
    setup(ctx, scene_from(spt, golden_scenes, "random"), W, H, 2, 12, seed=5)
    assert ctx.stats()["prim_list_blocks"] == 0
    g = np.zeros(W * H * 3, np.uint8)
    got = ctx.render_segment(y0, y1, x0, x1, g_data=g)
    osc = oscene_from(oracle, golden_scenes, "random")
    fr = oracle.make_frame(spt.camera_basis(EYE, LOOK, UP), EYE, SKY, W, H, 2, 12, 5)
    gw = np.zeros_like(g)
    want, _ = oracle.render_segment(osc, fr, y0, y1, x0, x1, rgb8=gw)
    assert_bitwise(got[:, :3], want[:, :3], f"{W}x{H} region")
    assert np.array_equal(g, gw)


def test_setters_rebuild_lists_only_when_they_change(spt, golden_scenes):
    """The primary-ray candidate lists depend on the accel tables, the camera and the frame
    size only: spp / depth / seed setters and a repeated camera keep them."""
    c = spt.Context(0)
    try:
        view = spt.camera_basis(EYE, LOOK, UP)
        c.set_scene(scene_from(spt, golden_scenes, "random"))
        c.set_camera(view, EYE, SKY)
        c.set_params(320, 200, 4, 50, 1)
        st = c.stats()
        assert st["prim_list_builds"] == 1 and st["prim_list_blocks"] > 0 and st["accel_build_ms"] > 0
        before = c.render_segment(0, 200, 0, 320)
        c.set_params(320, 200, 8, 20, 7)
        c.set_params(320, 200, 4, 50, 1)
        c.set_camera(view, EYE, SKY)
        assert c.stats()["prim_list_builds"] == 1
        assert_bitwise(c.render_segment(0, 200, 0, 320), before, "after setters that keep the lists")
        c.set_params(321, 200, 4, 50, 1)
        assert c.stats()["prim_list_builds"] == 2
        c.set_camera(spt.camera_basis([0.5, 1.2, -3, 0], LOOK, UP), [0.5, 1.2, -3, 0], SKY)
        assert c.stats()["prim_list_builds"] == 3
        c.set_scene(scene_from(spt, golden_scenes, "random"))
        assert c.stats()["prim_list_builds"] == 4
    finally:
        c.close()


@pytest.mark.parametrize("task", [False, True])
def test_config2_500_sphere_scene_region_vs_oracle(spt, ctx, oracle, task):
    """BASELINE.json config 2's "~500-sphere" RTIOW scene: GenerateSpheres with its rows run
    to z < 37.5 (488 spheres, uint32 index; SceneGenerators.hpp:32-53, Collision.hpp:87-92
    cap the reference at 255).  A 1200 x 800 frame's regions (one across the horizon with
    the far rows of small spheres, one on the big balls) at 8 spp, depth 50, against the
    oracle, float bits and g_data bytes; whichever walk the tree's size selects."""
    s = spt.generate_spheres(1, z_end=37.5)
    assert 480 <= s.n <= 520
    view = spt.camera_basis()
    ctx.set_scene(s)
    ctx.set_camera(view, spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
    ctx.set_params(1200, 800, 8, 50, 1)
    osc = oracle.OracleScene(s.centers, s.radii, s.colors, s.materials, s.fuzz)
    fr = oracle.make_frame(view, spt.scene.DEFAULT_EYE, spt.INIT_COLOR, 1200, 800, 8, 50, 1)
    for (y0, y1, x0, x1) in ((360, 400, 560, 680), (500, 540, 200, 260)):
        g = np.zeros(1200 * 800 * 3, np.uint8)
        got = ctx.render_segment(y0, y1, x0, x1, g_data=g, task=task)
        gw = np.zeros_like(g)
        want, _ = oracle.render_segment(osc, fr, y0, y1, x0, x1, rgb8=gw, task=task)
        if task and (y1 - y0) != (x1 - x0):
            same_bits_or_nan(got[:, :3], want[:, :3], f"500 spheres task {y0},{x0}")
        else:
            assert_bitwise(got[:, :3], want[:, :3], f"500 spheres {y0},{x0}")
        assert np.array_equal(g, gw)
