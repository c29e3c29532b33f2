"""CPU tests: the C-ABI library loads, exports what include/spt_hip.h declares,
and its host-only entry points behave (no GPU compute here)."""
import ctypes

import numpy as np
import pytest


def test_library_exports_every_declared_symbol(native):
    names = native.declared_symbols()
    assert len(names) >= 20
    L = native.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.spt_abi_version() == native.ABI_VERSION == 11


def test_ctx_create_reports_no_device_without_gpu(native):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = native.lib().spt_ctx_create(0, ctypes.byref(h))
    assert rc == 5  # SPT_ERR_NODEVICE
    assert native.lib().spt_last_error(None)
    assert not h.value


def test_null_context_is_an_argument_error(native):
    L = native.lib()
    assert L.spt_set_params(None, 10, 10, 1, 1, 1) == 1
    assert L.spt_render_segment(None, 0, 1, 0, 1, None, None) == 1
    assert b"null" in L.spt_last_error(None)


def test_tile_transport_validates_arguments(native):
    """spt_tiles_* (the copy-engine tile transport) reject a null context or transport
    before touching a device, and destroying a null transport is a no-op.  (The size,
    rank and side checks need a context, i.e. a GPU: tests/test_gpu_parity.py.)"""
    L = native.lib()
    h = ctypes.c_void_p()
    assert L.spt_tiles_create(None, b"x", 0, 2, 16, 2, ctypes.byref(h)) == 1
    assert not h.value
    assert L.spt_tiles_buffer(None, 0, ctypes.byref(h)) == 1
    assert L.spt_tiles_send_async(None, 0, None, None) == 1
    assert L.spt_tiles_recv_async(None, 0, None) == 1
    assert L.spt_tiles_release_async(None, 0, None) == 1
    assert L.spt_tiles_attach(None, None) == 1
    L.spt_tiles_destroy(None)
    assert b"null" in L.spt_last_error(None)


@pytest.mark.parametrize("h,strip,parts", [(800, 8, 1), (800, 8, 2), (800, 8, 3), (2160, 8, 8), (101, 4, 8),
                                           (7, 16, 4), (1, 1, 8)])
def test_row_split_partitions_the_frame(native, h, strip, parts):
    from simplepathtracer_amd import rows_count
    total = sum(rows_count(0, h, strip, parts, p) for p in range(parts))
    assert total == h
    # the row map of the kernel, restated: every y owned exactly once
    owner = np.full(h, -1)
    for p in range(parts):
        for k in range(rows_count(0, h, strip, parts, p)):
            blk = k // strip
            y = (blk * parts + p) * strip + (k - blk * strip)
            assert 0 <= y < h and owner[y] == -1
            owner[y] = p
    assert (owner >= 0).all()


def test_scene_generators_validate_arguments(native):
    L = native.lib()
    assert L.spt_scene_generate_random(1, 2, None, None, None, None, None, None) == 1
    import simplepathtracer_amd as spt
    s = spt.generate_stress(3, 1000)
    assert s.n == 1000 and (s.radii > 0).all() and set(np.unique(s.materials)) <= {1, 2, 3}
    c = spt.cornell3()
    assert c.n == 4 and list(c.materials) == [3, 3, 1, 2]


@pytest.mark.parametrize("w,h,parts", [(1200, 800, 8), (1200, 800, 3), (800, 1200, 5), (64, 8, 7), (3, 900, 4),
                                        (7, 5, 1)])
def test_task_ranges_partition_the_frame(native, w, h, parts):
    """spt_task_range (the rank-share split of a non-square task-mode frame): the parts'
    output ranges are contiguous and cover [0, W H) in order; the outputs that have sources
    (below W + (H - 1) H) are dealt evenly, the last part also takes the source-less tail."""
    from simplepathtracer_amd.renderer import task_range
    rs = [task_range(w, h, parts, r) for r in range(parts)]
    assert rs[0][0] == 0 and rs[-1][1] == w * h
    assert all(rs[k][1] == rs[k + 1][0] for k in range(parts - 1))
    n_src = min(w * h, w + (h - 1) * h)
    L = -(-n_src // parts)
    for r, (a, b) in enumerate(rs[:-1]):
        assert b - a == max(0, min(L, n_src - a)), (r, a, b)
    L_ = native.lib()
    x, y = ctypes.c_uint32(), ctypes.c_uint32()
    assert L_.spt_task_range(w, h, parts, parts, ctypes.byref(x), ctypes.byref(y)) == 1
    assert L_.spt_render_task_range_async(None, 0, 1, None, None) == 1


def test_wider_random_scene_extends_the_reference_rows(native):
    """spt_scene_generate_random_rows (BASELINE.json's "~500-sphere" scene): GenerateSpheres'
    row loop (SceneGenerators.hpp:32-53) run to z < 37.5 instead of 20 draws the same
    stream, so its first spheres are the reference-sized scene's, in order; every added
    sphere lies in the added rows; z_end 20 is spt_scene_generate_random itself; a bad
    z_end or a capacity below the scene is an argument error.  (Fuzz is drawn after the
    rows, so it differs.)"""
    import simplepathtracer_amd as spt
    a, b = spt.generate_spheres(1), spt.generate_spheres(1, z_end=37.5)
    assert a.n == 149 and 480 <= b.n <= 520
    for k in ("centers", "radii", "colors", "materials"):
        assert np.array_equal(getattr(b, k)[:a.n], getattr(a, k)), k
    assert (b.centers[a.n:, 2] >= 20.0).all() and (b.centers[a.n:, 2] < 37.5 + 0.3).all()
    c = spt.generate_spheres(1, z_end=20.0)
    for k in ("centers", "radii", "colors", "materials", "fuzz"):
        assert np.array_equal(getattr(c, k), getattr(a, k)), k
    L = native.lib()
    buf = [np.zeros(4 * 600, np.float32), np.zeros(600, np.float32), np.zeros(4 * 600, np.float32),
           np.zeros(600, np.uint8), np.zeros(600, np.float32)]
    n = ctypes.c_uint32()
    ptrs = [x.ctypes.data for x in buf]
    assert L.spt_scene_generate_random_rows(1, ctypes.c_float(-1.0), 600, *ptrs, ctypes.byref(n)) == 1
    assert L.spt_scene_generate_random_rows(1, ctypes.c_float(37.5), 300, *ptrs, ctypes.byref(n)) == 1
    assert L.spt_scene_generate_random_rows(1, ctypes.c_float(37.5), 600, *ptrs, ctypes.byref(n)) == 0
    assert n.value == b.n


def _build_shim_harness(tmp_path):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "simplepathtracer_amd", "lib")
    exe = str(tmp_path / "dropin_harness")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-pthread", f"-I{root}/include",
                    os.path.join(root, "tools", "dropin_harness.cpp"), f"-L{lib}", "-lspt_hip",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


def test_cpp_dropin_shim_compiles_against_the_c_abi(native, tmp_path):
    """include/spt/RenderSegmentShim.hpp + include/spt_hip.h build with plain g++
    (no HIP headers) in a translation unit shaped like the reference's."""
    import os
    assert os.path.exists(_build_shim_harness(tmp_path))


def _accel_check(native, centers, radii, k, b):
    P = ctypes.c_void_p
    c = np.ascontiguousarray(centers, np.float32)
    r = np.ascontiguousarray(radii, np.float32)
    nodes = ctypes.c_uint32(0)
    rc = native.lib().spt_accel_check(c.ctypes.data_as(P), r.ctypes.data_as(P), len(r), k, b, ctypes.byref(nodes))
    return rc, nodes.value, native.lib().spt_last_error(None)


@pytest.mark.parametrize("k,b", [(8, 0), (4, 0), (2, 0), (8, 2), (8, 4), (8, 16), (3, 4), (5, 0), (1, 2), (0, 4)])
@pytest.mark.parametrize("scene", ["random", "stress2000", "stress10000"])
def test_traversal_tables_are_valid(native, scene, k, b):
    """The culling tree's exactness rests on host-built tables: every sphere in
    exactly one slot, sound preorder/skip links in all 8 octant layouts, every flat
    node's bounding sphere and every tree node's expanded box containing all members
    below it (spt_accel.cpp validate_accel)."""
    import simplepathtracer_amd as spt
    s = spt.generate_spheres(1) if scene == "random" else spt.generate_stress(2, int(scene[6:]))
    rc, nodes, err = _accel_check(native, s.centers, s.radii, k, b)
    assert rc == 0, err
    if k == 0:
        assert nodes == 0  # brute force: every sphere in the always-list
    elif b == 0:
        assert nodes == -(-(s.n - 4) // k)  # flat: one node per cluster (4 big spheres are "always")
    else:
        assert nodes > -(-(s.n - 4) // k)


@pytest.mark.parametrize("case", ["empty", "tiny", "coincident", "nonfinite", "huge_spread", "beyond_1e15"])
def test_traversal_tables_edge_scenes(native, case):
    rng = np.random.default_rng(7)
    if case == "empty":
        c, r = np.zeros((0, 4)), np.zeros(0)
    elif case == "tiny":
        c, r = rng.normal(size=(5, 4)), np.full(5, 0.3)
    elif case == "coincident":  # every centre identical: degenerate Morton keys and Rb = r
        c, r = np.ones((300, 4)), np.full(300, 0.2)
    elif case == "nonfinite":  # non-finite spheres go to the always-list, never into a bound
        c, r = rng.normal(size=(400, 4)) * 10, rng.uniform(0.1, 0.3, 400)
        c[17, 1] = np.inf
        r[33] = np.nan
        c[90, 0] = np.nan
    elif case == "huge_spread":  # bounds spanning 1e-3 .. 1e5
        c = np.concatenate([rng.normal(size=(200, 4)) * 1e-3, rng.normal(size=(200, 4)) * 1e5])
        r = np.concatenate([np.full(200, 1e-4), np.full(200, 10.0)])
    else:  # members past 1e15 from the origin: their tree boxes are everything (never cull)
        c = np.concatenate([rng.normal(size=(300, 4)), rng.normal(size=(300, 4)) * 1e16])
        r = np.full(600, 0.2)
    for k, b in ((8, 0), (8, 4), (2, 2)):
        rc, _, err = _accel_check(native, c, r, k, b)
        assert rc == 0, (case, k, b, err)
    rc, _, _ = _accel_check(native, c, r, 9, 0)
    assert rc == 1


def test_item_orders_are_bijections(tmp_path):
    """The kernel's item orders -- [band][8x8 tile][sample][pixel] (spt::ts_item,
    the default) and [sample][8x8 tile][pixel] (spt::tile_pixel) -- cover every
    (sample, pixel) of any region exactly once; compiled for the host with hipcc."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "tile_check"
    subprocess.run(["hipcc", "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    "-I", os.path.join(root, "simplepathtracer_amd", "csrc"), "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "tile_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout


@pytest.mark.parametrize("w,h", [(4, 3), (5, 2), (1, 1), (7, 6)])
def test_save_bmp_matches_stb_layout(native, tmp_path, w, h):
    """io::SaveImage (IOHelpers.hpp:24-27) calls stbi_write_bmp(path, w, h, 3, g_data);
    stb is an absent submodule, so the expected file is built here from stb's published
    24-bit layout (stbi_write_bmp_core): 54-byte header, rows last-to-first, BGR,
    rows zero-padded to 4 bytes (parity unpinned against stb itself)."""
    import struct
    rng = np.random.default_rng(w * 10 + h)
    data = rng.integers(0, 256, w * h * 3, dtype=np.uint8)
    path = tmp_path / "out.bmp"
    P = ctypes.c_void_p
    assert native.lib().spt_save_bmp(str(path).encode(), w, h, 3, data.ctypes.data_as(P)) == 0
    pad = (-w * 3) & 3
    rows = [data[(h - 1 - r) * w * 3:(h - r) * w * 3].reshape(w, 3)[:, ::-1].tobytes() + b"\0" * pad
            for r in range(h)]
    body = b"".join(rows)
    header = b"BM" + struct.pack("<IHHI", 54 + len(body), 0, 0, 54) + \
        struct.pack("<IiiHHIIiiII", 40, w, h, 1, 24, 0, 0, 0, 0, 0, 0)
    assert path.read_bytes() == header + body
    assert native.lib().spt_save_bmp(str(path).encode(), w, h, 4, data.ctypes.data_as(P)) != 0
