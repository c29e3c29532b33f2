#!/bin/bash
# Service timeline A/B: variants x N (tools/svc_timeline.py), 2 reps each, wall only.
for v in "libspt_hip.so" "libspt_hip_ahead1.so" "libspt_hip_rq4.so" "libspt_hip_rq32.so" "libspt_hip.so SPT_SVC_CLAIM=896"; do
  set -- $v
  L=$1; shift
  for n in 8 1; do
    r=$(env SPT_LIB=$L "$@" timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms" | tr '\n' ' ')
    echo "$v n=$n: $r"
  done
done
for n in 8 1; do
  r=$(timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 --service 0 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms" | tr '\n' ' ')
  echo "no service n=$n: $r"
done
