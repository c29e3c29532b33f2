#!/bin/bash
# Steady-state cost of the service kernel's parts (timing only): N = 1 timelines of
# variants built with `make variants` (tools/svc_timeline.py, slope = ms per frame).
for v in "libspt_hip.so" "libspt_hip_plain.so" "libspt_hip.so SPT_SVC_CLAIM=896"; do
  set -- $v
  L=$1; shift
  r=$(env SPT_LIB=$L "$@" timeout -k 10 120 python tools/svc_timeline.py --n 1 --reps 2 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame" | tr '\n' ' ')
  echo "$v: $r"
done
r=$(timeout -k 10 120 python tools/svc_timeline.py --n 1 --reps 2 --service 0 2>&1 | grep -o "wall [0-9.]* ms\|slope [0-9.]* ms/frame" | tr '\n' ' ')
echo "launches: $r"
