#!/bin/bash
# The C++ drop-in's cold frame (one frame per process, Renderer.hpp:335-344), diagnosed:
# per-tile RenderJob spans (SPT_HARNESS_COLD=2) with the default library, without the
# tiling read-ahead's arming, without batching; then a kernel trace of the default run.
# Usage (GPU box): bash tools/cold_probe.sh <out_dir>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/${1:-gpurun_out/cold}
mkdir -p "$OUT"
H="$R/simplepathtracer_amd/lib/spt_dropin_harness"
for v in default SPT_BATCH_SETS=1 SPT_BATCH=0; do
  for rep in 1 2; do
    echo "== $v rep $rep"
    if [ "$v" = default ]; then
      SPT_HARNESS_COLD=2 timeout -k 10 120 "$H" /dev/null 1200 800 100 50 4 0 0 || exit $?
    else
      env "$v" SPT_HARNESS_COLD=2 timeout -k 10 120 "$H" /dev/null 1200 800 100 50 4 0 0 || exit $?
    fi
  done
done
cd /tmp && export TMPDIR=/tmp
SPT_HARNESS_COLD=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$H" /dev/null 1200 800 100 50 4 0 0
