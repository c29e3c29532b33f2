#!/bin/bash
# rocprofv3 kernel trace + PMC passes of a bench command (GPU box), then the SPT_DIAG
# build's in-kernel lane counts for the same config.
# Usage: tools/profile.sh <tag> <config> [bench args...]
#   e.g. tools/profile.sh r02_c2 c2            (the driver's default bench command)
#        tools/profile.sh r02_c5 c5 --config c5 --steps 2 --warmup 1 --no-cpu-baseline
# Every --pmc pass is its own run (rocprofv3 does not split counters over passes).
# A pass whose counter this rocprofv3 does not know fails fast and is skipped; a
# timeout, abort or fault ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-prof}
CFG=${2:-c2}
[ $# -ge 2 ] && shift 2 || shift $#
ARGS="$*"
[ -z "$ARGS" ] && ARGS="--no-dropin --no-cpu-baseline"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
step() {  # name fatal(0|1) timeout cmd...
  local name=$1 fatal=$2 t=$3; shift 3
  echo "== $name"
  timeout -k 10 -s KILL "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log"
  case $rc in 0) ;; 124|134|137|139) echo "stopping: $name rc=$rc"; exit $rc ;;
    *) [ "$fatal" = 1 ] && exit $rc ;; esac
  return 0
}
step trace 1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS
i=0
for group in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" \
             "SQC_DCACHE_HITS SQC_DCACHE_MISSES" \
             "FETCH_SIZE" "WRITE_SIZE" "VALUUtilization" "VALUBusy" "MeanOccupancyPerCU"; do
  i=$((i + 1))
  step pmc$i 0 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$R/bench.py" $ARGS
done
# the SPT_DIAG library is built beforehand on the build host (make -C simplepathtracer_amd/csrc diag)
[ -f "$R/simplepathtracer_amd/lib/libspt_hip_diag.so" ] || { echo "missing libspt_hip_diag.so"; exit 3; }
SPT_LIB=libspt_hip_diag.so step diag 1 300 python3 "$R/tools/diag.py" "$CFG" --json "$OUT/diag.json"
find "$OUT" -name "*.csv" | head -40
