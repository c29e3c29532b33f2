"""Where do blocks run under a CU mask?  (Reserved CUs)  Prints, per XCC,
the CUs a CU-masked stream's blocks land on, and where/when a collective-sized block
(512 threads, 256 VGPRs) queued on another stream beside a reserved-CU render starts.
Usage (GPU box): python tools/cu_mask_probe.py [--reserve 8]"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reserve", default="8,32", help="reserved-CU counts to probe")
ap.add_argument("--spp", type=int, default=400)
args = ap.parse_args()
lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simplepathtracer_amd", "lib")
h = ctypes.CDLL(os.path.join(lib, "libspt_testhooks.so"))
h.spt_test_where.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
h.spt_test_masked_stream.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
h.spt_test_stream_destroy.argtypes = [ctypes.c_void_p]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print(f"CUs {ncu}", flush=True)


def decode(w):
    w = w.reshape(-1, 4).astype(np.int64)
    hw, xcc = w[:, 0], w[:, 1] & 0xF
    cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7
    t = w[:, 2] | (w[:, 3] << 32)
    return xcc, se, sh, cu, t


def placement(stream, blocks, big, us=300):
    where = torch.zeros(blocks * 4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert h.spt_test_where(stream, us, blocks, big, where.data_ptr()) == 0
    torch.cuda.synchronize()
    return decode(where.cpu().numpy().view(np.uint32))


def per_xcc(xcc, se, sh, cu):
    out = {}
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        out[x] = sorted(set(zip(se[m].tolist(), sh[m].tolist(), cu[m].tolist())))
    return out


full = per_xcc(*placement(None, 4096, 0)[:4])
print("unmasked: " + " ".join(f"xcc{x}:{len(v)}" for x, v in full.items()), flush=True)
reserves = [int(x) for x in args.reserve.split(",")]
for res in reserves:
    ms = ctypes.c_void_p()
    assert h.spt_test_masked_stream(ncu - res, ncu, ctypes.byref(ms)) == 0
    masked = per_xcc(*placement(ms, 4096, 0)[:4])
    print(f"mask keep {ncu - res}: " + " ".join(f"xcc{x}:{len(v)}" for x, v in masked.items()), flush=True)
    for x in full:
        miss = sorted(set(full[x]) - set(masked.get(x, [])))
        print(f"  xcc{x} excluded (se, sh, cu): {miss}", flush=True)
    h.spt_test_stream_destroy(ms)

# a reserved-CU render on stream a; a collective-sized kernel on stream b just after it
W, H = 1200, 800
ctx = spt.Context(0)
ctx.set_scene(spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, args.spp, 50, 1)
a, b = torch.cuda.Stream(), torch.cuda.Stream()
rgba = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
for n in [0] + [r for r in reserves for _ in (0, 1)]:
    ctx.set_reserved_cus(n)
    where = torch.zeros(8 * 4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e0, er, eb = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(a)
    ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, rgba.data_ptr(), 0, a.cuda_stream)
    er.record(a)
    time.sleep(0.002)  # the render's blocks are resident before the probe is queued
    b.wait_event(e0)
    assert h.spt_test_where(ctypes.c_void_p(b.cuda_stream), 1000, 8, 1, where.data_ptr()) == 0
    eb.record(b)
    torch.cuda.synchronize()
    xcc, se, sh, cu, t = decode(where.cpu().numpy().view(np.uint32))
    print(f"reserve {n}: render {e0.elapsed_time(er):.2f} ms, probe ends {e0.elapsed_time(eb):.2f} ms; blocks at "
          + " ".join(f"x{a_}/se{b_}/sh{c_}/cu{d_}@{(tt - t.min()) / 100:.0f}us"
                     for a_, b_, c_, d_, tt in zip(xcc, se, sh, cu, t)), flush=True)
ctx.close()
