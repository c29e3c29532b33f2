#!/bin/bash
# Round-2 GPU-box session: GPU tests, smoke, the default bench line, other configs,
# rocprofv3 profiles (+ diag counts) of config 2 and config 5.
# Usage: tools/session_r2.sh "<steps>"   steps from: tests smoke bench c5 c3 c1 prof_c2 prof_c5
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
STEPS=${1:-"tests smoke bench"}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
for s in $STEPS; do
  case $s in
    tests) run gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_c2 400 python bench.py ;;
    c1) run bench_c1 200 python bench.py --config c1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    c3) run bench_c3 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline ;;
    c5) run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    prof_c2) run profile_c2 900 bash tools/profile.sh r02_c2 c2 ;;
    prof_c5) run profile_c5 900 bash tools/profile.sh r02_c5 c5 --config c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
