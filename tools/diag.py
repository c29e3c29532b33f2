"""Diagnostic run: in-kernel counters of the SPT_DIAG build (never used for timing).
Usage on the GPU box: SPT_LIB=libspt_hip_diag.so python tools/diag.py [config]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import simplepathtracer_amd as spt  # noqa: E402

args = [a for a in sys.argv[1:]]
json_out = None
if "--json" in args:
    k = args.index("--json")
    json_out = args[k + 1]
    del args[k:k + 2]
cfg = args[0] if args else "c2"
W, H, spp, b = {"c2": (1200, 800, 100, 50), "c2s": (1200, 800, 8, 50), "c5": (1920, 1080, 256, 50),
                "c5s": (1920, 1080, 4, 50), "c3": (3840, 2160, 1024, 50)}[cfg]
if len(args) > 1:  # bounces override (1: casts are almost all primary rays)
    b = int(args[1])
ctx = spt.Context(0)
scene = spt.generate_stress(1, 10000) if cfg.startswith("c5") else spt.generate_spheres(1)
ctx.set_scene(scene)
ctx.set_camera(spt.camera_basis(), spt.scene.DEFAULT_EYE, spt.INIT_COLOR)
ctx.set_params(W, H, spp, b, 1)
ctx.render_segment(0, H, 0, W)
ctx.reset_stats()
ctx.render_segment(0, H, 0, W)
st = ctx.stats()
it, leaves, nodes, cc, cs, cr, pairs, live = st["diag"][:8]
print(f"casts={st['casts']} samples={st['samples']} wave_iters={it} live_lanes/iter={st['casts']/max(it,1):.2f}")
k = os.environ.get("SPT_CLUSTER_K", "auto")
print(f"per wave cast: tree nodes tested={nodes/max(it,1):.2f} clusters entered={leaves/max(it,1):.2f} "
      f"(cluster size {k}, tree {os.environ.get('SPT_TREE_B', 'auto')})")
tot = max(cc + cs + cr, 1)
print(f"cycle shares: cast {cc/tot:.3f} shade {cs/tot:.3f} refill+ballot {cr/tot:.3f}")
print(f"(lane, cluster) pairs that may pass per cast={pairs/max(st['casts'],1):.2f}; "
      f"lane efficiency of entered clusters={pairs/max(live,1):.3f}")
sph, br, pas, imp = st["diag"][8:12]
print(f"per wave cast: spheres tested={sph/max(it,1):.2f} update branches taken={br/max(it,1):.2f} "
      f"({br/max(sph,1):.3f} of tested); lanes passing per taken branch={pas/max(br,1):.2f}; "
      f"taken branches where some lane improves its winner={imp/max(br,1):.3f}")
lt, lp = st["diag"][12:14]
print(f"lane-level RaySphereIntersection evaluations per ray={lt/max(st['casts'],1):.2f} "
      f"member pretests per ray={lp/max(st['casts'],1):.2f} (brute force: {scene.n})")
pi, pn, ps_, pb, pc = st["diag"][14:19]
if pi:
    print(f"primary batches: {pi} of {it} wave iterations ({pi/max(it,1):.3f}); per primary cast: nodes={pn/pi:.2f} "
          f"spheres={ps_/pi:.2f} update branches={pb/pi:.2f}; per other cast: nodes={(nodes-pn)/max(it-pi,1):.2f} "
          f"spheres={(sph-ps_)/max(it-pi,1):.2f} update branches={(br-pb)/max(it-pi,1):.2f}; "
          f"primary casts' share of cast cycles {pc/max(cc,1):.3f}")
scalls, srounds = st["diag"][19:21]
if scalls:
    print(f"sampler: {scalls} calls ({scalls/max(it,1):.3f} per wave iteration), {srounds/scalls:.3f} cooperative "
          f"rounds per call after round 0")
l8, l16, scyc = st["diag"][21:24]
if leaves:
    print(f"tree leaves entered by <= 8 lanes: {l8/leaves:.3f}, by <= 16 lanes: {l16/leaves:.3f}; "
          f"sampler cycles {scyc/max(cc + cs + cr, 1):.3f} of the phases' total")
ti, tlv = st["diag"][24:26]
if ti:
    print(f"drain (items run out): {ti} wave iterations ({ti/max(it,1):.4f} of all), {tlv/ti:.2f} live lanes per iteration")
print(f"render_ms={st['render_ms']:.3f}")
print("raw diag", list(st["diag"]))
# the LDS kernel (1024-thread blocks) walks lane by lane (spt_path.h find_closest_lane):
# nodes = lane node visits, live = walk iterations, leaves = leaf passes, pairs = lane leaf tests
lane_walk = st["block_threads"] == 1024
if lane_walk:
    print(f"lane walk: node visits per ray={nodes/max(st['casts'],1):.2f} walk iterations per wave cast="
          f"{live/max(it,1):.2f} leaf passes per wave cast={leaves/max(it,1):.2f} leaves per ray="
          f"{pairs/max(st['casts'],1):.2f} lane leaves per leaf pass={pairs/max(leaves,1):.2f}")
if json_out:
    import json
    json.dump({"config": cfg, "frame": [W, H, spp, b], "spheres": scene.n, "casts": st["casts"],
               "samples": st["samples"], "lane_tests_per_ray": lt / max(st["casts"], 1),
               "lane_pretests_per_ray": lp / max(st["casts"], 1), "clusters_entered_per_wave_cast": leaves / max(it, 1),
               "tree_nodes_per_wave_cast": nodes / max(it, 1), "live_lanes_per_iter": st["casts"] / max(it, 1),
               "wave_iters": it, "spheres_per_wave_cast": sph / max(it, 1), "update_branches_per_wave_cast": br / max(it, 1),
               "cycle_split": {"cast": cc / tot, "shade": cs / tot, "refill": cr / tot},
               "primary": {"iters": pi, "nodes_per_cast": pn / max(pi, 1), "spheres_per_cast": ps_ / max(pi, 1),
                           "update_branches_per_cast": pb / max(pi, 1), "cast_cycle_share": pc / max(cc, 1)},
               "sampler": {"calls": scalls, "rounds_after_first_per_call": srounds / max(scalls, 1)},
               "build": "SPT_DIAG=1 (libspt_hip_diag.so), counters only, never timed",
               **({"walk": "lane", "lane_node_visits_per_ray": nodes / max(st["casts"], 1),
                   "walk_iters_per_wave_cast": live / max(it, 1), "leaf_passes_per_wave_cast": leaves / max(it, 1),
                   "leaves_per_ray": pairs / max(st["casts"], 1), "lane_leaves_per_leaf_pass": pairs / max(leaves, 1),
                   "note": "lane walk: clusters_entered/tree_nodes per wave cast count leaf passes and lane "
                           "node visits"} if lane_walk else {"walk": "wave"})}, open(json_out, "w"), indent=1)
