"""Timeline of a rocprofv3 kernel trace (run_kernel_trace.csv): per spt kernel its
launches' durations, and over the traced span the time covered by >= 1 render launch,
by >= 2, and the gaps with none.  Usage: python tools/trace_timeline.py <trace.csv> [last_n]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "spt::" in r["Kernel_Name"]]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
renders = [x for x in iv if "render" in x[2]]
if last:
    renders = renders[-last:]
t0, t1 = renders[0][0], max(x[1] for x in renders)
ev = sorted([(a, 1) for a, _, _ in renders] + [(b, -1) for _, b, _ in renders])
cover = {0: 0, 1: 0, 2: 0}
depth, prev = 0, t0
for t, d in ev:
    cover[min(depth, 2)] += t - prev
    depth += d
    prev = t
span = t1 - t0
print(f"render launches {len(renders)} over {span / 1e6:.3f} ms: none {cover[0] / 1e6:.3f} ms, "
      f"one {cover[1] / 1e6:.3f} ms, two+ {cover[2] / 1e6:.3f} ms")
d = sorted((b - a) / 1e6 for a, b, _ in renders)
print(f"render launch ms: min {d[0]:.3f} median {d[len(d) // 2]:.3f} max {d[-1]:.3f} sum {sum(d):.3f}")
folds = [(b - a) / 1e6 for a, b, k in iv if "fold" in k and a >= t0]
if folds:
    folds.sort()
    print(f"fold launches {len(folds)}: median {folds[len(folds) // 2]:.3f} ms max {folds[-1]:.3f} ms")
for a, b, k in renders[:12]:
    print(f"  {k:40s} start {(a - t0) / 1e6:8.3f} end {(b - t0) / 1e6:8.3f} ({(b - a) / 1e6:.3f})")
