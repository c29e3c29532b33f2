"""Summarize a tools/profile.sh output directory into profiles/<name>.md
(kernel-trace stats + per-kernel PMC averages, FETCH_SIZE corrected x2 per
MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
timed = int(sys.argv[3]) if len(sys.argv) > 3 else 20  # bench --steps of the profiled run
cmd = sys.argv[4] if len(sys.argv) > 4 else "(default arguments)"
out = [f"# rocprofv3 summary: {os.path.basename(src)}\n",
       "Command: `tools/profile.sh` = rocprofv3 --kernel-trace --stats and separate --pmc passes (one counter "
       "group each) over "
       f"`python3 bench.py {cmd}` (1x MI355X).\n",
       "## Kernel trace (--kernel-trace --stats)\n", "| kernel | calls | avg ms | min ms | max ms | % |",
       "|---|---|---|---|---|---|"]
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    out.append(f"| `{r['Name'][:60]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
               f"{float(r['MinNs'])/1e6:.4f} | {float(r['MaxNs'])/1e6:.4f} | {float(r['Percentage']):.2f} |")
# the timed launches only (the last `timed` of each spt kernel): clocks ramp over the
# warmup launches, and bench.py's HIP-event average covers the timed ones.  The render
# service's kernel (render_kernel_svc) is one dispatch per session: its timed session is
# its last dispatch, which renders all `timed` frames (per-frame figures = / timed).
SVC = "render_kernel_svc"
trace = os.path.join(src, "trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        if "spt::" in r["Kernel_Name"]:
            per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out += ["", f"## Timed launches (last {timed} per kernel, from run_kernel_trace.csv)\n",
            "Span = a dispatch's own start-to-end time.  With frames in flight two render launches "
            "run at once (the next frame fills the CUs while the previous one drains), so spans overlap; "
            "`union/launch` = length of the union of the timed launches' intervals / launches, the device "
            "time per launch that bench.py's roofline uses (from its HIP events).\n",
            "| kernel | launches | avg span ms | min ms | max ms | union/launch ms |", "|---|---|---|---|---|---|"]
    for k, v in sorted(per.items()):
        iv = sorted((x[0], x[0] + x[1]) for x in v)[-(1 if SVC in k else timed):]
        d = [(b - a) / 1e6 for a, b in iv]
        tot, cs, ce = 0, None, None
        for a, b in iv:
            if ce is None or a > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        tot += ce - cs
        out.append(f"| `{k[:60]}` | {len(d)} | {sum(d)/len(d):.4f} | {min(d):.4f} | {max(d):.4f} | "
                   f"{tot/1e6/len(d):.4f} |")
        if SVC in k:
            out.append(f"| `{k[:60]}` per frame | {timed} frames in the last session | "
                       f"{sum(d)/timed:.4f} | | | {tot/1e6/timed:.4f} |")
agg = collections.defaultdict(list)
for d in sorted(x for x in os.listdir(src) if x.startswith("pmc")):
    p = os.path.join(src, d, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        if "spt::" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])].append(
                (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
# the timed dispatches only (the last `timed` of each kernel, as in the trace section): the
# bench's probe render (one row) and warmup frames would otherwise pull the average down
# the service's last session renders `timed` frames: per-frame values of the extensive
# counters (instructions, cycles, bytes); ratios and means stay as measured
INTENSIVE = ("VALUUtilization", "VALUBusy", "MeanOccupancyPerCU")
for key, v in agg.items():
    if SVC in key[0]:
        agg[key] = [x if key[1] in INTENSIVE else x / timed for _, x in sorted(v)[-1:]]
    else:
        agg[key] = [x for _, x in sorted(v)[-timed:]]
out += ["", f"## PMC counters (average per dispatch over the last {timed} dispatches of each kernel; for "
        f"{SVC}: its last dispatch / {timed} frames, i.e. per frame; separate passes)\n",
        "| kernel | counter | value |", "|---|---|---|"]
for (k, c), v in sorted(agg.items()):
    val = sum(v) / len(v)
    note = ""
    # rocprofv3 reports both in KiB (1024 bytes); printed in decimal megabytes (1e6 bytes)
    if c == "FETCH_SIZE":
        note = f" (KiB; x2 gfx950 correction = {2*val*1024/1e6:,.1f} MB, decimal)"
    elif c == "WRITE_SIZE":
        note = f" (KiB = {val*1024/1e6:,.1f} MB, decimal)"
    out.append(f"| `{k}` | {c} | {val:,.0f}{note} |")
open(dst, "w").write("\n".join(out) + "\n")
# profiles/counters.json[config]: per-launch PMC values of the render and fold kernels
# (FETCH_SIZE x2 gfx950 correction, KB -> bytes; derived VALU/occupancy figures) and
# the SPT_DIAG lane counts (diag.json of tools/profile.sh) that bench.py reports in
# roofline.traffic and roofline_valu; SPT_COUNTERS_CONFIG names the config
ccfg = os.environ.get("SPT_COUNTERS_CONFIG")
if ccfg:
    import json
    cp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "counters.json")
    doc = json.load(open(cp)) if os.path.exists(cp) else {}
    rel = os.path.relpath(os.path.abspath(dst), os.path.dirname(os.path.dirname(os.path.abspath(cp))))
    entry = {}
    for short in ("render_kernel", "fold_kernel"):
        # the render kernel of the timed frames: the service's when it ran (the bench's
        # one-row probe launch is a plain render_kernel dispatch)
        names = {k for (k, c) in agg if short in k}
        if short == "render_kernel" and any(SVC in k for k in names):
            names = {k for k in names if SVC in k}
        vals = {c: sum(v) / len(v) for (k, c), v in agg.items() if k in names}
        if not vals:
            continue
        e = {"source": rel}
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            e["fetch_bytes"] = int(2 * vals["FETCH_SIZE"] * 1024)
            e["write_bytes"] = int(vals["WRITE_SIZE"] * 1024)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVES", "SQ_ACTIVE_INST_VALU",
                  "SQ_THREAD_CYCLES_VALU", "SQC_DCACHE_HITS", "SQC_DCACHE_MISSES", "VALUUtilization", "VALUBusy",
                  "MeanOccupancyPerCU"):
            if c in vals:
                e[c] = round(vals[c], 4) if vals[c] < 1e4 else int(vals[c])
        if "VALUUtilization" not in e and "SQ_THREAD_CYCLES_VALU" in vals and vals.get("SQ_ACTIVE_INST_VALU"):
            e["VALUUtilization"] = round(100 * vals["SQ_THREAD_CYCLES_VALU"] / (vals["SQ_ACTIVE_INST_VALU"] * 64), 2)
        if "MeanOccupancyPerCU" in vals:
            e["occupancy_waves_per_simd"] = round(vals["MeanOccupancyPerCU"] / 4, 3)
        if vals.get("SQC_DCACHE_HITS") is not None and vals.get("SQC_DCACHE_MISSES") is not None:
            tot = vals["SQC_DCACHE_HITS"] + vals["SQC_DCACHE_MISSES"]
            e["sqc_dcache_miss_frac"] = round(vals["SQC_DCACHE_MISSES"] / tot, 4) if tot else None
        entry[short] = e
    dj = os.path.join(src, "diag.json")
    if os.path.exists(dj):
        d = json.load(open(dj))
        d["source"] = rel
        entry["diag"] = d
    doc[ccfg] = entry
    json.dump(doc, open(cp, "w"), indent=2)
print("\n".join(out))
