#!/bin/bash
# The C++ drop-in's cold frame (one frame per process, Renderer.hpp:335-344): three cold
# runs per mode, then one under rocprofv3 with the HIP API, kernel and copy traces, which
# show where the frame's host calls wait (round 6: the first device-to-host hipMemcpy2D
# of a process took 8.6 ms; spt_prepare_dropin now pays it at context creation).
# Usage (GPU box): bash tools/cold_api_trace.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 2
R=$(pwd)
TAG=${1:-cold}
H=$R/simplepathtracer_amd/lib/spt_dropin_harness
mkdir -p gpurun_out
for i in 1 2 3; do
  for task in 0 1; do
    SPT_HARNESS_COLD=1 timeout -k 5 30 "$H" /dev/null 1200 800 100 50 4 $task 0 2>&1 | tail -1 || exit $?
  done
done
(cd /tmp && export TMPDIR=/tmp && SPT_HARNESS_COLD=2 timeout -k 10 120 rocprofv3 --hip-runtime-trace --kernel-trace \
   --memory-copy-trace --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run -- "$H" /dev/null 1200 800 100 50 4 0 0 \
   > "$R/gpurun_out/${TAG}_trace.log" 2>&1) || exit $?
tail -1 "gpurun_out/${TAG}_trace.log"
