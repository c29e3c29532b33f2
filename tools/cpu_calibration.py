import sys, time
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
import numpy as np, pyoracle as po
import simplepathtracer_amd.scene as sc
import simplepathtracer_amd as spt
scene = spt.generate_spheres(1)
view = spt.camera_basis()
osc = po.OracleScene(scene.centers, scene.radii, scene.colors, scene.materials, scene.fuzz)
for mode in (0, 1):
    fr = po.make_frame(view, [0,1,-3,0], [137,207,240,0], 1200, 800, 100, 50, 1)
    t=time.perf_counter(); po.render_image_parallel(osc, fr, 16, mode=mode, want_rgba=False); dt=time.perf_counter()-t
    print("mode", mode, "N", scene.n, "sec", round(dt,2), "Msamples/s", round(1200*800*100/dt/1e6,3), flush=True)
