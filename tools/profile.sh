#!/bin/bash
# rocprofv3 kernel-trace + PMC passes of a short bench run (GPU box).
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-prof}; shift || true
# default: the driver's own bench command (python bench.py, config 2, two frames in flight)
ARGS=${@:-""}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS
step pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc1" -o run -- python3 "$R/bench.py" $ARGS
step pmc_busy 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc2" -o run -- python3 "$R/bench.py" $ARGS
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3" -o run -- python3 "$R/bench.py" $ARGS
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc4" -o run -- python3 "$R/bench.py" $ARGS
find "$OUT" -name "*.csv" | head -40
