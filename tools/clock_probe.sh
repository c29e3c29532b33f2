#!/bin/bash
# Clock and power of the GPU while config-2 frames render back to back (launched, two
# streams, ~40 s): rocm-smi / amd-smi samples every 2 s from 15 s in.
# Usage (GPU box): bash tools/clock_probe.sh [reserve_cus]
set -o pipefail
mkdir -p gpurun_out
RES=${1:-0}
(timeout -k 10 90 python -u - "$RES" > gpurun_out/r05k_loop.log 2>&1 <<'PY'
import sys, time, torch
import simplepathtracer_amd as spt
W, H = 1200, 800
c = spt.Context(0)
c.set_scene(spt.generate_spheres(1))
c.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
c.set_params(W, H, 100, 50, 1)
c.set_reserved_cus(int(sys.argv[1]))
st = [torch.cuda.Stream(), torch.cuda.Stream()]
buf = [torch.zeros((W * H, 4), device="cuda") for _ in st]
t0 = time.time(); k = 0; last = t0
while time.time() - t0 < 40:
    for _ in range(50):
        c.render_rows_async(0, 0, H, 1, 1, 0, 0, W, buf[k % 2].data_ptr(), 0, st[k % 2].cuda_stream); k += 1
    torch.cuda.synchronize()
    if time.time() - last > 2:
        print(f"{time.time() - t0:6.1f} s: {k} frames, {W * H * 100 * k / (time.time() - t0) / 1e6:8.0f} Msamples/s", flush=True)
        last = time.time()
PY
) &
BP=$!
sleep 15
for i in 1 2 3 4 5; do timeout -k 5 20 amd-smi metric -p -c -t >> gpurun_out/r05k_amdsmi.log 2>&1; sleep 2; done
wait $BP
