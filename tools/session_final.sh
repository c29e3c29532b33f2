#!/bin/bash
# GPU-box measurement session: GPU tests, smoke, the default bench line, the other
# configs at full size, the rocprofv3 profile of the default bench, diag counters.
# Usage: tools/session_final.sh <profile tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run gpu_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c2 300 python bench.py
run bench_c1 200 python bench.py --config c1 --steps 20 --warmup 3
run bench_c3 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline
run bench_c5 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline
bash tools/profile.sh "${1:-prof}" c2 > gpurun_out/profile.log 2>&1 || { tail gpurun_out/profile.log; exit 3; }
make -s -C simplepathtracer_amd/csrc diag > gpurun_out/diag_build.log 2>&1 || exit 3
SPT_LIB=libspt_hip_diag.so run diag_c2 200 python tools/diag.py c2
