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
       "Command: `tools/profile.sh` = rocprofv3 --kernel-trace --stats and four separate --pmc passes over "
       f"`python3 bench.py {cmd}` (1x MI355X).\n",
       "## Kernel trace (--kernel-trace --stats)\n", "| kernel | calls | avg ms | min ms | max ms | % |",
       "|---|---|---|---|---|---|"]
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
    out.append(f"| `{r['Name'][:60]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
               f"{float(r['MinNs'])/1e6:.4f} | {float(r['MaxNs'])/1e6:.4f} | {float(r['Percentage']):.2f} |")
# the timed launches only (the last `timed` of each spt kernel): clocks ramp over the
# warmup launches, and bench.py's HIP-event average covers the timed ones
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
        iv = sorted((x[0], x[0] + x[1]) for x in v)[-timed:]
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
agg = collections.defaultdict(list)
for d in ("pmc1", "pmc2", "pmc3", "pmc4"):
    p = os.path.join(src, d, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        if "spt::" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
out += ["", "## PMC counters (average per dispatch, separate passes)\n", "| kernel | counter | value |", "|---|---|---|"]
for (k, c), v in sorted(agg.items()):
    val = sum(v) / len(v)
    note = ""
    if c == "FETCH_SIZE":
        note = f" (KB; x2 gfx950 correction = {2*val/1024:.1f} MB)"
    elif c == "WRITE_SIZE":
        note = f" (KB = {val/1024:.1f} MB)"
    out.append(f"| `{k}` | {c} | {val:,.0f}{note} |")
open(dst, "w").write("\n".join(out) + "\n")
# profiles/traffic.json: HBM bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
# KB -> bytes) that bench.py reports as roofline.traffic; SPT_TRAFFIC_CONFIG names the config
tcfg = os.environ.get("SPT_TRAFFIC_CONFIG")
if tcfg:
    import json
    tp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    doc = json.load(open(tp)) if os.path.exists(tp) else {}
    entry = {}
    for kname, short in (("render_kernel", "render_kernel"), ("fold_kernel", "fold_kernel")):
        f = [sum(v) / len(v) for (k, c), v in agg.items() if short in k and c == "FETCH_SIZE"]
        w = [sum(v) / len(v) for (k, c), v in agg.items() if short in k and c == "WRITE_SIZE"]
        if f and w:
            entry[kname] = {"fetch_bytes": int(2 * f[0] * 1024), "write_bytes": int(w[0] * 1024),
                            "source": os.path.relpath(os.path.abspath(dst), os.path.dirname(os.path.dirname(os.path.abspath(tp))))}
    doc[tcfg] = entry
    json.dump(doc, open(tp, "w"), indent=2)
print("\n".join(out))
