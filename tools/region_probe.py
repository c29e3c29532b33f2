"""Fixed-cost probe: render-kernel device time for config-2 regions of growing
height (full width, 100 spp), to separate the per-launch intercept from the
per-sample slope.  Usage (GPU box): python tools/region_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402

W, H, SPP, B = 1200, 800, 100, 50
ctx = spt.Context(0)
ctx.set_scene(spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, SPP, B, 1)
out = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
spp_env = os.environ.get("SPT_PROBE_SPP")
for rows in (1, 8, 32, 104, 200, 400, 800):
    ts, rs = [], []
    for r in range(4):
        ctx.reset_stats()
        y0 = 400 - rows // 2
        ctx.render_rows_async(spt.MODE_SEGMENT, y0, y0 + rows, 1, 1, 0, 0, W, out.data_ptr(), 0, 0)
        ctx.synchronize()
        st = ctx.stats()
        if r:
            ts.append(st["render_ms"])
            rs.append(st["casts"])
    t = float(np.median(ts))
    print(f"rows {rows:4d}: samples {rows * W * SPP / 1e6:8.2f} M  render {t:8.3f} ms  "
          f"{rows * W * SPP / t / 1e6:8.1f} Msamples/s  rays/sample {rs[0] / (rows * W * SPP):.3f}", flush=True)
