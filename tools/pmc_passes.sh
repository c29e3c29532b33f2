#!/bin/bash
# Several rocprofv3 --pmc passes (one counter group each) over a short c2 bench
# run with one library build; prints render-kernel averages per dispatch.
# Usage: tools/pmc_passes.sh tag lib.so "CNT_A CNT_B ..." "CNT_C ..." ...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1 LIB=$2; shift 2
cd /tmp && export TMPDIR=/tmp
i=0
for group in "$@"; do
  i=$((i + 1))
  out="$R/gpurun_out/$TAG/pass$i"
  mkdir -p "$out"
  SPT_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$out" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$out/log" 2>&1 || exit $?
done
python3 - "$R/gpurun_out/$TAG" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spt::render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):16,.0f}")
PY
