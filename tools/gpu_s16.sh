#!/bin/bash
# GPU session: tools/gpu_s15.sh (drop-in tests + drop-in A/B of $VARIANTS), then a
# render A/B of the library builds $KVARIANTS on $CONFIGS (tools/ab.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_s15.sh || exit $?
for c in ${CONFIGS:-c5}; do
  libs="libspt_hip.so"; for v in $KVARIANTS; do libs="$libs libspt_hip_$v.so"; done
  echo "== ab $c"
  timeout -k 10 400 python tools/ab.py $libs --rounds ${ROUNDS_K:-3} --config $c > gpurun_out/ab_$c.log 2>&1 || { tail -20 gpurun_out/ab_$c.log; exit 1; }
  grep "render ms" gpurun_out/ab_$c.log
done
