"""Summarize a tools/profile.sh output directory into profiles/<name>.md
(kernel-trace stats + per-kernel PMC averages, FETCH_SIZE corrected x2 per
MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
timed = int(sys.argv[3]) if len(sys.argv) > 3 else 12  # bench --steps of the profiled run
out = [f"# rocprofv3 summary: {os.path.basename(src)}\n",
       "Command: `tools/profile.sh` = rocprofv3 --kernel-trace --stats and four separate --pmc passes over "
       f"`python3 bench.py --steps {timed} --warmup 4 --no-cpu-baseline --streams 1` (config 2, 1x MI355X, one frame in flight so per-kernel durations are not stretched by overlap).\n",
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
            "| kernel | launches | avg ms | min ms | max ms |", "|---|---|---|---|---|"]
    for k, v in sorted(per.items()):
        d = [x[1] / 1e6 for x in sorted(v)][-timed:]
        out.append(f"| `{k[:60]}` | {len(d)} | {sum(d)/len(d):.4f} | {min(d):.4f} | {max(d):.4f} |")
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
print("\n".join(out))
