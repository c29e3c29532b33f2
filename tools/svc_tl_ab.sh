#!/bin/bash
# Service timeline A/B (tools/svc_timeline.py, 2 reps each): "LIB [ENV=VAL...]" variants x N,
# then launches.
for v in "libspt_hip.so" "libspt_hip_lag0.so"; do
  set -- $v
  L=$1; shift
  for n in 8 1; do
    r=$(env SPT_LIB=$L "$@" timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms\|Error.*" | tr '\n' ' ')
    echo "$v n=$n: $r"
  done
done
