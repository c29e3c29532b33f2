#!/bin/bash
# GPU session: the HEAD check (tests, smoke, config benches), then an interleaved A/B
# of $VARIANTS on $CONFIGS (tools/ab.py).  Every step bounded; a failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/session_check.sh || exit $?
for c in ${CONFIGS:-c5}; do
  libs="libspt_hip.so"; for v in $VARIANTS; do libs="$libs libspt_hip_$v.so"; done
  echo "== ab $c"
  timeout -k 10 400 python tools/ab.py $libs --rounds ${ROUNDS:-3} --config $c > gpurun_out/ab_$c.log 2>&1 || exit $?
  tail -n 8 gpurun_out/ab_$c.log
done
