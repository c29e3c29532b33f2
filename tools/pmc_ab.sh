#!/bin/bash
# PMC instruction counts of the render kernel for several library builds (GPU box).
# Usage: tools/pmc_ab.sh tag lib1.so lib2.so ...   (bench.py c2, 2 steps)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  out="$R/gpurun_out/$TAG/${lib%.so}"
  mkdir -p "$out"
  SPT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES --output-format csv -d "$out" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$out/log" 2>&1 || exit $?
  python3 - "$out" "$lib" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spt::render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: f"{sum(v)/len(v)/1e9:.3f}G" for k, v in sorted(agg.items())})
PY
done
