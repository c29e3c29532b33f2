"""profiles/<name>.md from tools/attrib.sh output directories (attrib.json): per-phase VALU
of the config-2 render kernel.  Usage: python tools/attrib_md.py <out.md> <label>=<attrib dir> ...
Rays and wave iterations per frame come from the SPT_DIAG build (tools/diag.py, same kernel)."""
import json
import os
import sys

RAYS, ITERS = 221314766, 3482444  # per config-2 frame (SPT_DIAG, profiles/r05_diag.txt)
ROWS = [("cast: whole FindClosestIntersectionSphere (list or tree walk, always-list, setup)", "libspt_hip_dup1.so"),
        ("  tree node tests (box slabs, near / front bounds)", "libspt_hip_dup8.so"),
        ("  member tests + closest-contact updates of entered leaves", "libspt_hip_dup16.so"),
        ("cube-minus-ball sampler (coop_ball_vector, splitmix draws)", "libspt_hip_dup2.so"),
        ("primary ray (start_path: keyed RNG, jitter, camera, normalize)", "libspt_hip_dup4.so"),
        ("  (of the cast) the always-tested group (ground, big balls)", "libspt_hip_dup32.so"),
        ("  (of the cast) the primary batches' candidate-list casts", "libspt_hip_dup64.so"),
        ("shading step less the sampler", "libspt_hip_dup128.so")]
dst = sys.argv[1]
out = ["# Per-phase VALU attribution of the config-2 render kernel (round 5)", "",
       "Method (`tools/attrib.sh`): one `rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES` pass per library over",
       "`bench.py --steps 4 --warmup 1 --service 0` (config 2, 1200x800x100, depth 50), averaged over the 5 frame launches",
       "(bench.py's one-row probe launch excluded).  The `SPT_DUP` builds (`spt_path.h`) run one phase a second time on",
       "opaque copies of its inputs and discard the copy, so the increase in instructions per launch is that phase's",
       "own count (plus a few register moves for the copies and any spill code the second copy causes).  The product",
       "kernel's instruction stream is unchanged by the switches (`tools/isa_regions.py --compare`).",
       f"Per frame: {RAYS:,} rays and {ITERS:,} wave iterations (SPT_DIAG counts).", ""]
for arg in sys.argv[2:]:
    label, _, d = arg.partition("=")
    res = json.load(open(os.path.join(d, "attrib.json")))
    V = res["libspt_hip.so"]["SQ_INSTS_VALU"]
    S = res["libspt_hip.so"]["SQ_INSTS_SALU"]
    out += [f"## {label} (`{d}`)", "",
            "| phase | VALU per frame | share | per wave iteration | lane-slots per ray | SALU per frame |",
            "|---|---|---|---|---|---|",
            f"| whole kernel (product build) | {V:,.0f} | 1.000 | {V / ITERS:.0f} | {V * 64 / RAYS:.0f} | {S:,.0f} |"]
    dv = {}
    for name, lib in ROWS:
        if lib not in res:
            continue
        dv[lib] = res[lib]["SQ_INSTS_VALU"] - V
        ds = res[lib]["SQ_INSTS_SALU"] - S
        out.append(f"| {name} | {dv[lib]:,.0f} | {dv[lib] / V:.3f} | {dv[lib] / ITERS:.0f} | {dv[lib] * 64 / RAYS:.0f} | {ds:,.0f} |")
    rc = dv["libspt_hip_dup1.so"] - dv["libspt_hip_dup8.so"] - dv["libspt_hip_dup16.so"]
    rest = V - dv["libspt_hip_dup1.so"] - dv["libspt_hip_dup2.so"] - dv["libspt_hip_dup4.so"]
    out.append(f"| (cast less nodes and leaves: always-list, candidate-list casts, per-cast setup) | {rc:,.0f} | "
               f"{rc / V:.3f} | {rc / ITERS:.0f} | {rc * 64 / RAYS:.0f} | |")
    out.append(f"| (rest: shading step less sampler, refill / claims / queue, loop control) | {rest:,.0f} | "
               f"{rest / V:.3f} | {rest / ITERS:.0f} | {rest * 64 / RAYS:.0f} | |")
    out += ["", "Raw averages per library:", "", "```", json.dumps(res, indent=1), "```", ""]
open(dst, "w").write("\n".join(out) + "\n")
print("\n".join(out[:40]))
