#!/bin/bash
# GPU session: GPU tests of the current build, then interleaved A/B (tools/ab.py) of
# libspt_hip.so against $VARIANTS on $CONFIGS.  Usage: VARIANTS="base r8" tools/gpu_prim.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  echo "== gpu tests"
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -n 3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-c2}; do
  libs="libspt_hip.so"; for v in $VARIANTS; do libs="$libs libspt_hip_$v.so"; done
  echo "== ab $c"
  timeout -k 10 400 python tools/ab.py $libs --rounds ${ROUNDS:-4} --config $c || exit $?
done
