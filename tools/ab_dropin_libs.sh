#!/bin/bash
# A/B of library builds on the drop-in path: the C++ shim under RenderImageParallelMain
# tiling (tools/dropin_harness.cpp, config 2), libspt_hip.so against each entry of
# $VARIANTS -- `v` for libspt_hip_v.so, `name@VAR=VAL` for libspt_hip.so with that
# environment -- interleaved over $ROUNDS rounds, tc in $TCS, segment (and task with TASK=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=simplepathtracer_amd/lib
mkdir -p gpurun_out
names="main"
for v in $VARIANTS; do names="$names $v"; done
for n in $names; do
  lib=${n%%@*}
  d=gpurun_out/dropin_$lib; mkdir -p $d
  cp $L/spt_dropin_harness $d/
  case $lib in main|*=*) cp $L/libspt_hip.so $d/ ;; *) [ -f $L/libspt_hip_$lib.so ] && cp $L/libspt_hip_$lib.so $d/libspt_hip.so || cp $L/libspt_hip.so $d/ ;; esac
done
for r in $(seq ${ROUNDS:-3}); do
  for n in $names; do
    lib=${n%%@*}; env=""; [ "$n" != "$lib" ] && env=${n#*@} && env=${env//,/ }
    for tc in ${TCS:-4}; do
      for task in 0 ${TASK:+1}; do
        res=$(env $env timeout -k 10 120 gpurun_out/dropin_$lib/spt_dropin_harness /dev/null 1200 800 100 50 $tc $task 5) || exit $?
        sec=${res#*seconds=}; sec=${sec%% *}
        python3 -c "print('round $r $n tc=$tc task=$task', round(1200*800*100*5/$sec/1e6, 1), 'Msamples/s')"
      done
    done
  done
done
rm -rf gpurun_out/dropin_*
