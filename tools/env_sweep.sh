#!/bin/bash
# bench.py (config 2, 40 timed frames, no CPU baseline / drop-in legs) once per
# environment setting, interleaved over two rounds; prints value per setting.
# Usage (GPU box): tools/env_sweep.sh TAG "VAR=A" "VAR=B" ...   ("-" = defaults)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
mkdir -p "$R/gpurun_out/$TAG"
for r in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    log="$R/gpurun_out/$TAG/s${i}_r$r.log"
    if [ "$setting" = "-" ]; then
      timeout -k 10 120 python3 "$R/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --no-dropin > "$log" 2>&1
    else
      timeout -k 10 120 env $setting python3 "$R/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --no-dropin > "$log" 2>&1
    fi
    rc=$?
    [ $rc -eq 0 ] || { echo "$setting rc=$rc"; exit $rc; }
    echo "$setting round $r: $(grep -o '"value": [0-9.]*' "$log")"
  done
done
