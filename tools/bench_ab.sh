#!/bin/bash
# Interleaved bench.py A/B of library builds: libspt_hip.so against libspt_hip_$v.so for v
# in $VARIANTS, $ROUNDS rounds, bench arguments $ARGS (default: config 2, no drop-in / CPU legs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for v in main $VARIANTS; do
    lib=libspt_hip.so; [ $v != main ] && lib=libspt_hip_$v.so
    SPT_LIB=$lib timeout -k 10 200 python bench.py ${ARGS:---no-dropin --no-cpu-baseline} | python3 -c "import json,sys; d=json.loads([x for x in sys.stdin if x.startswith('{')][-1]); print('round $r $v', d['value'], d['ms_per_step'])" || exit $?
  done
done
