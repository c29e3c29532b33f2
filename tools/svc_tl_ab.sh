#!/bin/bash
# Service timeline A/B (tools/svc_timeline.py, 2 reps each): env variants x N, then launches.
for v in "SPT_SVC_X=0" "SPT_SVC_TAIL_CLAIM=0" "SPT_SVC_TAIL_DIV=4" "SPT_SVC_TAIL_CLAIM=64" "SPT_SVC_CLAIM=448"; do
  for n in 8 1; do
    r=$(env $v timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms" | tr '\n' ' ')
    echo "$v n=$n: $r"
  done
done
for n in 8 1; do
  r=$(timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 --service 0 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms" | tr '\n' ' ')
  echo "launches n=$n: $r"
done
