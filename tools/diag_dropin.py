"""Diagnose drop-in shim mismatches: run tools/dropin_harness (built in-tree) for one
tile grid, with and without SPT_DEVICES, and compare with tile renders through the
Python context; prints mismatch counts per tile."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import simplepathtracer_amd as spt  # noqa: E402

exe = os.path.join(ROOT, "simplepathtracer_amd", "lib", "spt_dropin_harness")
w, h, spp, tc = 1200, 800, 6, int(sys.argv[1]) if len(sys.argv) > 1 else 8
golden = dict(np.load(os.path.join(ROOT, "tests", "golden", "scenes.npz"), allow_pickle=False))
from test_gpu_parity import scene_from, setup  # noqa: E402
c = spt.Context(0)
setup(c, scene_from(spt, golden, "random"), w, h, spp, 50)
want = np.zeros(w * h * 3, np.uint8)
sw, sh = w // tc, h // tc
for j in range(tc):
    for i in range(tc):
        c.render_segment(sh * j, sh * j + sh, sw * i, sw * i + sw, want)
c.close()
for devs in (None, "0,0"):
    env = dict(os.environ)
    if devs:
        env["SPT_DEVICES"] = devs
    out = "/tmp/gd.bin"
    r = subprocess.run([exe, out, str(w), str(h), str(spp), "50", str(tc), "0"], env=env, capture_output=True, text=True)
    got = np.fromfile(out, np.uint8)
    bad = np.nonzero(got != want)[0]
    print(f"devices={devs} rc={r.returncode} bad bytes={bad.size}", r.stdout.strip()[-200:])
    if bad.size:
        px = bad // 3
        y = h - 1 - px // w
        x = px % w
        tiles = sorted(set(zip((y // sh).tolist(), (x // sw).tolist())))
        print("  tiles:", tiles[:40], "n", len(tiles))
        print("  first", list(zip(y[:5].tolist(), x[:5].tolist())), got[bad[:5]], want[bad[:5]])
