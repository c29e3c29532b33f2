#!/bin/bash
# Launch-path claim size A/B on the config-2 bench line (SPT_CLAIM), interleaved rounds.
B="python bench.py --no-cpu-baseline --no-dropin --service 0"
for r in 1 2; do
  for c in "" 640 896 1344; do
    v=$(SPT_CLAIM=$c timeout -k 10 120 $B 2>&1 | grep -o '"value": [0-9.]*')
    echo "r$r claim=${c:-auto}: $v"
  done
done
