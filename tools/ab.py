"""Interleaved A/B timing of render-kernel variants in ONE process.
Usage: python tools/ab.py libspt_hip_g4.so libspt_hip_g8.so ... [--rounds 5] [--config c2]
Each variant is its own ctypes CDLL (RTLD_LOCAL) over the same C ABI."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+", help="lib.so[:cluster_k[:tree_branching]][@VAR=VAL,...] (env at ctx creation)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--config", default="c2")
ap.add_argument("--mode", type=int, default=0)
args = ap.parse_args()
torch.cuda.init()
from simplepathtracer_amd import _native  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402

W, H, SPP, B = {"c1": (200, 100, 4, 8), "c2": (1200, 800, 100, 50), "c2x10": (1200, 800, 1000, 50),
                "c2hi": (2400, 1600, 25, 50), "c3s": (3840, 2160, 16, 50),
                "c5": (1920, 1080, 256, 50), "c5x2": (1920, 1080, 512, 50), "c2x2": (1200, 800, 200, 50),
                "c5s": (1920, 1080, 4, 50), "s20k": (1920, 1080, 16, 50), "s30k": (1920, 1080, 16, 50), "s40k": (1920, 1080, 16, 50),
                "s50k": (1920, 1080, 16, 50), "c2w": (1200, 800, 100, 50)}[args.config]
scene = (spt.generate_stress(1, int(args.config[1:3]) * 1000) if args.config in ("s20k", "s30k", "s40k", "s50k") else spt.generate_stress(1, 10000) if args.config.startswith("c5")
         else spt.cornell3() if args.config == "c1" else spt.generate_spheres(1, z_end=37.5) if args.config == "c2w"
         else spt.generate_spheres(1))
view = spt.camera_basis()
P = ctypes.c_void_p
ctxs = []
for name in args.libs:
    spec, _, envs = name.partition("@")
    for kv in filter(None, envs.split(",")):
        var, _, val = kv.partition("=")
        os.environ[var] = val
    libname, _, rest = spec.partition(":")
    ck, _, tb = rest.partition(":")
    for var, val in (("SPT_CLUSTER_K", ck), ("SPT_TREE_B", tb)):
        if val:
            os.environ[var] = val
        else:
            os.environ.pop(var, None)
    L = ctypes.CDLL(os.path.join(ROOT, "simplepathtracer_amd", "lib", os.path.basename(libname)))
    L.spt_ctx_create.argtypes = [ctypes.c_int, P]
    L.spt_set_scene.argtypes = [P, P, P, P, P, P, ctypes.c_uint32]
    L.spt_set_camera.argtypes = [P, P, P, P]
    L.spt_set_params.argtypes = [P] + [ctypes.c_uint32] * 4 + [ctypes.c_uint64]
    L.spt_render_rows_async.argtypes = [P, ctypes.c_int] + [ctypes.c_uint32] * 7 + [P, P, P]
    L.spt_get_stats.argtypes = [P, P]
    L.spt_reset_stats.argtypes = [P]
    L.spt_synchronize.argtypes = [P]
    h = P()
    assert L.spt_ctx_create(0, ctypes.byref(h)) == 0
    q = lambda a: a.ctypes.data_as(P)
    assert L.spt_set_scene(h, q(scene.centers), q(scene.radii), q(scene.colors), q(scene.materials),
                           q(scene.fuzz), scene.n) == 0
    e = np.float32(spt.scene.DEFAULT_EYE); sk = np.float32(spt.INIT_COLOR)
    assert L.spt_set_camera(h, q(view), q(e), q(sk)) == 0
    assert L.spt_set_params(h, W, H, SPP, B, 1) == 0
    ctxs.append((name, L, h))
    for kv in filter(None, envs.split(",")):
        os.environ.pop(kv.partition("=")[0], None)
frames = {name: torch.zeros((H * W, 4), dtype=torch.float32, device="cuda") for name, _, _ in ctxs}
res = {name: [] for name, _, _ in ctxs}
for r in range(args.rounds + 1):
    for name, L, h in ctxs:
        L.spt_reset_stats(h)
        assert L.spt_render_rows_async(h, args.mode, 0, H, 1, 1, 0, 0, W, P(frames[name].data_ptr()), None, None) == 0
        assert L.spt_synchronize(h) == 0
        st = _native.Stats()
        assert L.spt_get_stats(h, ctypes.byref(st)) == 0
        if r:
            res[name].append(st.render_ms)
ref = frames[ctxs[0][0]].view(torch.int32)
for name, _, _ in ctxs:
    same = torch.equal(frames[name].view(torch.int32), ref)
    v = np.array(res[name])
    print(f"{name:28s} render ms median {np.median(v):8.3f} min {v.min():8.3f}  "
          f"Msamples/s {W*H*SPP/np.median(v)/1e3:9.1f}  identical={same}")
