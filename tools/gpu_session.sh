#!/bin/bash
# One GPU-box session: build, GPU tests, smoke, bench.  Stops at the first step
# that fails (LENIENT=1: only at a fault / abort / timeout, not a pytest failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-tests smoke bench}"
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 3; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  # any failure stops the session (LENIENT=1: only faults / aborts / timeouts do)
  if [ $rc -ne 0 ] && { [ -z "$LENIENT" ] || [ $rc -ne 1 ]; }; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    alltests) run gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    *) run custom 900 bash -c "$s" ;;
  esac
done
