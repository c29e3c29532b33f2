#!/bin/bash
# GPU session: kernel traces of the C++ drop-in at tc = 4 (config 2, 3 frames) with the
# default batch grid and with SPT_BATCH_GRID_DIV=1, each summarized by trace_timeline.py
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for div in 2 1; do
  OUT="$R/gpurun_out/tdrop$div"; mkdir -p "$OUT"
  SPT_BATCH_GRID_DIV=$div timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    "$R/simplepathtracer_amd/lib/spt_dropin_harness" /dev/null 1200 800 100 50 4 0 3 > "$OUT/run.log" 2>&1 || exit 1
  echo "== div $div: $(tail -n 1 $OUT/run.log)"
  python3 "$R/tools/trace_timeline.py" "$(find $OUT -name '*kernel_trace.csv' | head -1)" 48 || exit 1
done
