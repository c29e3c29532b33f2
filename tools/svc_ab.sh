#!/bin/bash
# A/B of render-service settings on the config-2 bench line and the 8-way share probe
# (GPU box; each run under its own limit; stops on a timeout or crash).
B="python bench.py --no-cpu-baseline --no-dropin"
run() {  # label, then env assignments and the command
  local label=$1; shift
  local out; out=$(env "$@" 2>&1 | grep -o '"value": [0-9.]*\|wall per frame *[0-9.]* ms' | tr '\n' ' ')
  local rc=${PIPESTATUS[0]}
  echo "$label: $out"
}
for r in 1 2; do
  run "r$r svc0" timeout -k 10 120 $B --service 0
  run "r$r svc1" timeout -k 10 120 $B --service 1
  run "r$r svc1 wt0" SPT_LIB=libspt_hip_wt0.so timeout -k 10 120 $B --service 1
  run "r$r svc1 claim896" SPT_SVC_CLAIM=896 timeout -k 10 120 $B --service 1
  run "r$r svc1 claim256" SPT_SVC_CLAIM=256 timeout -k 10 120 $B --service 1
done
P="python tools/scaling_probe.py --streams 2 --reps 3 --ns 8"
run "n8 svc0" timeout -k 10 120 $P --service 0
run "n8 svc1" timeout -k 10 120 $P --service 1
run "n8 svc1 wt0" SPT_LIB=libspt_hip_wt0.so timeout -k 10 120 $P --service 1
run "n8 svc1 claim256" SPT_SVC_CLAIM=256 timeout -k 10 120 $P --service 1
run "n8 svc1 claim896" SPT_SVC_CLAIM=896 timeout -k 10 120 $P --service 1
run "n8 svc0 strip8" timeout -k 10 120 $P --service 0 --strip 8
run "n8 svc1 strip8" timeout -k 10 120 $P --service 1 --strip 8
run "n8 svc1 strip20" timeout -k 10 120 $P --service 1 --strip 20
