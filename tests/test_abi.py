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
    assert L.spt_abi_version() == 1


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


def _build_shim_harness(tmp_path):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "simplepathtracer_amd", "lib")
    exe = str(tmp_path / "shim_harness")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", f"-I{root}/include",
                    os.path.join(root, "tests", "cpp", "shim_harness.cpp"), f"-L{lib}", "-lspt_hip",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


def test_cpp_dropin_shim_compiles_against_the_c_abi(native, tmp_path):
    """include/spt/RenderSegmentShim.hpp + include/spt_hip.h build with plain g++
    (no HIP headers) in a translation unit shaped like the reference's."""
    import os
    assert os.path.exists(_build_shim_harness(tmp_path))
