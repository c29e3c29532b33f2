#!/bin/bash
# GPU-box session: GPU tests, then interleaved A/B of the default library against
# the variants named in $VARIANTS (libspt_hip_<name>.so) on configs $CONFIGS.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1
rc=$?; tail -3 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2}; do
  libs="libspt_hip.so"; for v in $VARIANTS; do libs="$libs libspt_hip_$v.so"; done
  echo "== ab $c"
  timeout -k 10 300 python tools/ab.py $libs --rounds ${ROUNDS:-4} --config $c || exit $?
done
