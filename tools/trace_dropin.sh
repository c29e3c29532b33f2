# Kernel trace of the C++ drop-in at the shipped tc = 4 (config 2, 3 timed frames):
# launch start/end times of every render and fold, to see how the tiles' launches overlap.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/tdrop"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
  "$R/simplepathtracer_amd/lib/spt_dropin_harness" /dev/null 1200 800 100 50 4 0 ${TDROP_FRAMES:-3} > "$OUT/run.log" 2>&1
