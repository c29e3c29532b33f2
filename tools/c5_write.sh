#!/bin/bash
# C5 render WRITE_SIZE per launch against SPT_CLAIM (the slot write amplification,
# VERDICT r3 item 6).  GPU box; one PMC pass per setting.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for c in "" 128 512 1024; do
  d="$R/gpurun_out/c5w_${c:-def}"
  SPT_CLAIM=$c timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d" -o run -- \
    python3 "$R/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > "$d.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "claim ${c:-def}: rc=$rc"; exit $rc; }
  python3 - "$d" "${c:-def}" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
v = [float(r["Counter_Value"]) for r in rows if "render_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
print(f"claim {sys.argv[2]}: render launches {len(v)}, WRITE_SIZE per launch (last) {v[-1]:.0f} KiB-units; all {[round(x) for x in v]}")
PY
done
