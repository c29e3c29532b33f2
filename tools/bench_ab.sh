#!/bin/bash
# Interleaved bench.py A/B: libspt_hip.so against each entry of $VARIANTS -- `v` for
# libspt_hip_v.so, `name@VAR=VAL[,VAR=VAL]` for libspt_hip.so with that environment --
# $ROUNDS rounds, bench arguments $ARGS (default: config 2, no drop-in / CPU legs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${ROUNDS:-3}); do
  for v in main $VARIANTS; do
    lib=libspt_hip.so; env=""
    case $v in main) ;; *@*) env=${v#*@}; env=${env//,/ } ;; *) lib=libspt_hip_$v.so ;; esac
    env SPT_LIB=$lib $env timeout -k 10 200 python bench.py ${ARGS:---no-dropin --no-cpu-baseline} | python3 -c "import json,sys; d=json.loads([x for x in sys.stdin if x.startswith('{')][-1]); print('round $r $v', d['value'], d['ms_per_step'])" || exit $?
  done
done
