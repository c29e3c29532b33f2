"""Minimal service render (one frame through the render service, in-kernel fold on/off),
for diagnosing the service on the GPU box: prints the stats and compares with a launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import simplepathtracer_amd as spt  # noqa: E402

W, H, SPP = 320, 200, 16
ctx = spt.Context(0)
ctx.set_scene(spt.generate_spheres(1))
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, SPP, 50, 1)
ref = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
got = torch.zeros_like(ref)
ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, ref.data_ptr(), 0, 0)
ctx.synchronize()
print("launched ok", flush=True)
ctx.service_start()
ctx.render_rows_async(0, 0, H, 1, 1, 0, 0, W, got.data_ptr(), 0, 0)
print("published", flush=True)
ctx.service_stop()
ctx.synchronize()
st = ctx.stats()
print({k: st[k] for k in ("svc_sessions", "svc_jobs", "svc_inkernel_folds", "svc_running")}, flush=True)
same = torch.equal(got.view(torch.int32), ref.view(torch.int32))
print("identical:", same, flush=True)
ctx.close()
sys.exit(0 if same and st["svc_inkernel_folds"] == 1 else 1)
